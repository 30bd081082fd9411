"""Flash attention on the GPU beyond the BERT shape, each against an fp32 PyTorch reference:

* the benchmark shapes at their real sequence lengths: GPT-2 (S 1024, d 64, causal) and
  Megatron (S 2048, d 128, causal), with and without dropout (batch / heads reduced);
* head dims 32, 64, 128, 256 natively and 48 / 80 / 96 / 160 through zero padding;
* additive score biases (key padding [B,1,1,Sk], full [B,H,Sq,Sk], per-head [1,H,Sq,Sk]
  ALiBi-style, boolean masks) in forward AND backward, causal and not;
* dropout keep bits pinned to an independent Python Philox4x32-7 for sampled rows, so the mask
  generator itself is checked (not only its mean keep rate);
* the backward's QKV bias-gradient column sums (dsum) against the fp32 reference gradients.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(q, k, v, causal, scale, bias=None, mask=None, p=0.0, k_lens=None):
    """q, k, v [B, S, H, D] fp32 leaves -> o [B, Sq, H, D] (fp32)."""
    qf, kf, vf = (t.transpose(1, 2) for t in (q, k, v))
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    Sq, Sk = s.shape[-2], s.shape[-1]
    if bias is not None:
        s = s + bias.float()
    if causal:
        s = s.masked_fill(torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    if k_lens is not None:
        km = torch.arange(Sk, device=q.device)[None, :] >= k_lens[:, None].long()
        s = s.masked_fill(km[:, None, None, :], float("-inf"))
    pm = torch.nan_to_num(torch.softmax(s, -1))
    if mask is not None:
        pm = pm * mask.float() / (1.0 - p)
    return torch.matmul(pm, vf).transpose(1, 2)


def _check(qkv, o, do, dt, causal, scale, bias=None, mask=None, p=0.0, tol_scale=1.0):
    q, k, v = qkv.detach().float().unbind(2)
    qr, kr, vr = (t.clone().requires_grad_(True) for t in (q, k, v))
    orf = _ref(qr, kr, vr, causal, scale, bias=bias, mask=mask, p=p)
    orf.backward(do.float())
    tol = (2e-2 if dt == torch.bfloat16 else 5e-3) * tol_scale
    torch.testing.assert_close(o.float(), orf, rtol=tol, atol=tol)
    gtol = (5e-2 if dt == torch.bfloat16 else 1.5e-2) * tol_scale
    dq, dk, dv = qkv.grad.float().unbind(2)
    torch.testing.assert_close(dv, vr.grad, rtol=gtol, atol=gtol)
    torch.testing.assert_close(dk, kr.grad, rtol=gtol, atol=gtol)
    torch.testing.assert_close(dq, qr.grad, rtol=gtol, atol=gtol)
    return qr, kr, vr


# ----------------------------------------------------------------------------------- long shapes
@pytest.mark.parametrize("name,B,S,H,D", [("gpt2", 1, 1024, 2, 64), ("megatron", 1, 2048, 2, 128)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_benchmark_shapes(name, B, S, H, D, p):
    import apex._ext as e
    from apex.contrib.multihead_attn import flash

    C = e.require()
    dt = torch.bfloat16
    torch.manual_seed(7)
    qkv = (torch.randn(B, S, 3, H, D, device=DEV) * 0.5).to(dt).requires_grad_(True)
    scale = 1.0 / math.sqrt(D)
    torch.manual_seed(11)
    o = flash.flash_attention_packed(qkv, p, True, scale)
    mask = None
    if p > 0:
        torch.manual_seed(11)
        seed, offset = flash._seed_pair(p, qkv.device)
        mask = C.flash_dropout_mask(B, H, S, S, p, seed, offset, qkv.device)
    do = torch.randn_like(o)
    o.backward(do)
    _check(qkv, o, do, dt, True, scale, mask=mask, p=round(p * 256) / 256, tol_scale=1.5)


# ----------------------------------------------------------------------------------- head dims
@pytest.mark.parametrize("D", [32, 48, 64, 80, 96, 128, 160, 256])
@pytest.mark.parametrize("causal", [False, True])
def test_head_dims(D, causal):
    from apex.contrib.multihead_attn.attention import attention_packed

    dt = torch.bfloat16
    torch.manual_seed(D)
    B, S, H = 2, 160, 2
    qkv = (torch.randn(B, S, 3, H, D, device=DEV) * 0.7).to(dt).requires_grad_(True)
    scale = 1.0 / math.sqrt(D)
    o = attention_packed(qkv, None, 0.0, causal, scale)
    assert o.shape == (B, S, H, D)
    do = torch.randn_like(o)
    o.backward(do)
    _check(qkv, o, do, dt, causal, scale)


# ----------------------------------------------------------------------------------- biases
def _bias(kind, B, H, S, dt):
    g = torch.Generator(device=DEV).manual_seed(5)
    if kind == "key_padding":
        lens = torch.tensor([S, S // 2 + 3][:B], device=DEV)
        pad = torch.arange(S, device=DEV)[None, :] >= lens[:, None]
        return torch.zeros(B, 1, 1, S, device=DEV).masked_fill(pad[:, None, None, :], float("-inf")).to(dt)
    if kind == "full":
        return (torch.randn(B, H, S, S, device=DEV, generator=g) * 1.5).to(dt)
    if kind == "alibi":
        slopes = torch.tensor([2.0 ** -(i + 1) for i in range(H)], device=DEV)
        rel = torch.arange(S, device=DEV)[None, :] - torch.arange(S, device=DEV)[:, None]
        return (slopes[:, None, None] * rel[None].float())[None].to(dt)
    if kind == "bool":  # True = attend (SDPA convention); random sparsity, diagonal kept
        m = torch.rand(S, S, device=DEV, generator=g) > 0.3
        return m | torch.eye(S, dtype=torch.bool, device=DEV)
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["key_padding", "full", "alibi", "bool"])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("S,D", [(128, 64), (300, 64), (200, 128)])
def test_additive_bias(kind, causal, S, D):
    from apex.contrib.multihead_attn.attention import attention_packed

    dt = torch.bfloat16
    B, H = 2, 2
    torch.manual_seed(S + D)
    qkv = (torch.randn(B, S, 3, H, D, device=DEV) * 0.7).to(dt).requires_grad_(True)
    bias = _bias(kind, B, H, S, dt)
    scale = 1.0 / math.sqrt(D)
    o = attention_packed(qkv, bias, 0.0, causal, scale)
    do = torch.randn_like(o)
    o.backward(do)
    ref_bias = bias if bias.dtype != torch.bool else torch.zeros(bias.shape, device=DEV).masked_fill(~bias, float("-inf"))
    _check(qkv, o, do, dt, causal, scale, bias=ref_bias.float())


def test_bias_with_dropout_matches_masked_reference():
    import apex._ext as e
    from apex.contrib.multihead_attn import flash
    from apex.contrib.multihead_attn.attention import prepare_bias

    C = e.require()
    dt, B, S, H, D, p = torch.bfloat16, 2, 192, 2, 64, 0.2
    torch.manual_seed(1)
    qkv = (torch.randn(B, S, 3, H, D, device=DEV) * 0.7).to(dt).requires_grad_(True)
    bias = prepare_bias(_bias("full", B, H, S, dt), B, H, S, S, dt)
    torch.manual_seed(4)
    o = flash.flash_attention_packed(qkv, p, False, None, None, bias)
    torch.manual_seed(4)
    seed, offset = flash._seed_pair(p, qkv.device)
    mask = C.flash_dropout_mask(B, H, S, S, p, seed, offset, qkv.device)
    do = torch.randn_like(o)
    o.backward(do)
    _check(qkv, o, do, dt, False, 1.0 / math.sqrt(D), bias=bias.float(), mask=mask, p=round(p * 256) / 256)


# ----------------------------------------------------------------------------------- dropout bits
_M32 = 0xFFFFFFFF


def _philox4x32_7(seed, subseq, offset):
    key = [seed & _M32, (seed >> 32) & _M32]
    c = [offset & _M32, (offset >> 32) & _M32, subseq & _M32, (subseq >> 32) & _M32]
    for _ in range(7):
        p0 = 0xD2511F53 * c[0]
        p1 = 0xCD9E8D57 * c[2]
        hi0, lo0 = (p0 >> 32) & _M32, p0 & _M32
        hi1, lo1 = (p1 >> 32) & _M32, p1 & _M32
        c = [hi1 ^ c[1] ^ key[0], lo1, hi0 ^ c[3] ^ key[1], lo0]
        key = [(key[0] + 0x9E3779B9) & _M32, (key[1] + 0xBB67AE85) & _M32]
    return c


def _xorshift128_words(state, n):
    x, y, z, w = state
    out = []
    for _ in range(n):
        t = (x ^ (x << 11)) & _M32
        x, y, z = y, z, w
        w = (w ^ (w >> 19) ^ t ^ (t >> 8)) & _M32
        out.append(w)
    return out


def _keep_bits_python(seed, offset, bh, row, Sq, Sk, thresh):
    """Keep flag of every key of one attention row, the kernels' documented mapping: one stream per
    (row, half hl = bit 2 of the key) — a Philox4x32-7 call (counter offset + hl, subsequence
    bh * Sq + row) seeds xorshift128, each 32-key block takes the next 4 words — key k <-> byte k >> 3
    of word k & 3 of its half's block words, kept iff that byte >= thresh."""
    nblk = (Sk + 31) // 32
    streams = []
    for hl in (0, 1):
        st = _philox4x32_7(seed, bh * Sq + row, offset + hl)
        if not any(st):
            st[3] = 1
        streams.append(_xorshift128_words(st, 4 * nblk))
    keep = []
    for blk in range(nblk):
        for k in range(32):
            key = 32 * blk + k
            if key >= Sk:
                break
            w = streams[(k >> 2) & 1][4 * blk + (k & 3)]
            byte = (w >> (8 * (k >> 3))) & 0xFF
            keep.append(1 if byte >= thresh else 0)
    return keep


def test_dropout_mask_statistics():
    """The keep mask over a large [B*H, S, S] draw: keep rate at 1 - thresh/256 per key position and
    per row, and no correlation between neighbouring keys, neighbouring rows or the two halves of a
    block (each |corr| well below 1e-2 over ~10^7 pairs)."""
    import apex._ext as e

    C = e.require()
    B, H, S, p = 8, 16, 256, 0.1
    mask = C.flash_dropout_mask(B, H, S, S, p, 0xABCDEF, 0x1234, torch.device(DEV)).float().view(B * H, S, S)
    thresh = min(255, max(1, int(p * 256 + 0.5)))
    want = 1 - thresh / 256
    assert abs(float(mask.mean()) - want) < 2e-3
    assert float((mask.mean(dim=(0, 1)) - want).abs().max()) < 0.02  # every key position
    assert float((mask.mean(dim=2) - want).abs().max()) < 0.12  # every row (256 draws)
    z = mask - mask.mean()

    def corr(a, b):
        return float((a * b).mean() / (a.std() * b.std()))

    for a, b, what in ((z[..., 1:], z[..., :-1], "keys"), (z[:, 1:], z[:, :-1], "rows"),
                       (z[..., 4:], z[..., :-4], "halves"), (z[..., 32:], z[..., :-32], "blocks")):
        c = corr(a, b)
        assert abs(c) < 1e-2, (what, c)


@pytest.mark.parametrize("p", [0.1, 0.5])
def test_dropout_bits_match_python_stream(p):
    import apex._ext as e

    C = e.require()
    B, H, Sq, Sk = 2, 3, 37, 100
    seed, offset = 0x1234_5678_9ABC, 0x7777_0000_0011
    mask = C.flash_dropout_mask(B, H, Sq, Sk, p, seed, offset, torch.device(DEV)).cpu()
    thresh = min(255, max(1, int(p * 256 + 0.5)))
    for bh, row in [(0, 0), (1, 5), (5, 36), (3, 17)]:
        got = mask.view(B * H, Sq, Sk)[bh, row].tolist()
        assert got == _keep_bits_python(seed, offset, bh, row, Sq, Sk, thresh), (bh, row)
    assert abs(float(mask.float().mean()) - (1 - thresh / 256)) < 0.03


# ----------------------------------------------------------------------------------- dsum vs fp32
@pytest.mark.parametrize("S,causal", [(128, False), (200, True), (384, False)])
def test_dsum_against_fp32_reference(S, causal):
    """The backward's per-sequence column sums of dq, dk, dv (the packed QKV projection's bias
    gradient before the batch sum) against the fp32 reference gradients."""
    import apex._ext as e

    C = e.require()
    torch.manual_seed(S)
    B, H, D = 3, 4, 64
    qkv = (torch.randn(B, S, 3, H, D, device=DEV) * 0.7).bfloat16()
    q, k, v = qkv.unbind(2)
    scale = D ** -0.5
    o, lse, dmask = C.flash_attn_fwd(q, k, v, causal, scale, 0.0, 0, 0, None)
    do = torch.randn_like(o)
    dqkv = torch.empty_like(qkv)
    dq, dk, dv = dqkv.unbind(2)
    dsum = torch.zeros(B, 3 * H * D, device=DEV)
    C.flash_attn_bwd(do, q, k, v, o, lse, dq, dk, dv, causal, scale, 0.0, 0, 0, None, dmask, dsum)
    qr, kr, vr = (t.float().clone().requires_grad_(True) for t in qkv.unbind(2))
    _ref(qr, kr, vr, causal, scale).backward(do.float())
    ref = torch.stack([qr.grad, kr.grad, vr.grad], 2).sum(1).reshape(B, 3 * H * D)
    torch.testing.assert_close(dsum, ref, rtol=3e-2, atol=0.25)
