"""fp32 flash attention on the f32 MFMA (csrc/attention_f32.hip) against an fp64 reference of the
same op: forward output, log-sum-exp and all three input gradients, over head dims, causal masks,
odd and unequal lengths, per-batch key lengths, broadcast additive biases (with -inf entries) and
dropout (the reference applies the keep bits the kernel stored, and the bits themselves must be
the Philox/xorshift stream of the 16-bit kernels)."""
import math

import pytest
import torch

DEV = "cuda"


def _C():
    import apex._ext as e

    return e.require()


def _ref(q, k, v, do, scale, causal, k_lens=None, bias=None, keep=None, drop_scale=1.0):
    """fp64 reference: o, lse, dq, dk, dv; ``keep`` [B, H, Sq, Sk] 0/1."""
    q, k, v, do = (t.double().detach().requires_grad_(True) if i < 3 else t.double()
                   for i, t in enumerate((q, k, v, do)))
    B, Sq, H, D = q.shape
    Sk = k.shape[1]
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) * scale
    if bias is not None:
        s = s + bias.double()
    if k_lens is not None:
        km = torch.arange(Sk, device=q.device)[None, :] >= k_lens[:, None].long()
        s = s.masked_fill(km[:, None, None, :], float("-inf"))
    if causal:
        s = s.masked_fill(torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    lse = torch.logsumexp(s, -1)
    p = torch.exp(s - lse[..., None]).nan_to_num(0.0)
    if keep is not None:
        p = p * keep.double() * drop_scale
    o = torch.einsum("bhqk,bkhd->bqhd", p, v)
    o.backward(do)
    lse = torch.where(torch.isfinite(lse), lse, torch.full_like(lse, float("inf")))
    return o.detach(), lse.detach(), q.grad, k.grad, v.grad


def _run(q, k, v, do, scale, causal, p=0.0, k_lens=None, bias=None, seed=0, offset=0):
    C = _C()
    o, lse, dmask = C.flash_attn_fwd(q, k, v, causal, scale, p, seed, offset, k_lens, bias)
    dq, dk, dv = (torch.empty_like(t) for t in (q, k, v))
    C.flash_attn_bwd(do, q, k, v, o, lse, dq, dk, dv, causal, scale, p, seed, offset, k_lens, dmask, None, 0, bias)
    return o, lse, dq, dk, dv, dmask


def _keep_from_words(dmask, B, H, Sq, Sk):
    nblk = (Sk + 31) // 32
    w = dmask.view(torch.int32).view(B, H, Sq, nblk)
    bits = (w.unsqueeze(-1) >> torch.arange(32, device=w.device, dtype=torch.int32)) & 1
    return bits.reshape(B, H, Sq, nblk * 32)[..., :Sk]


def _check(got, ref, what, o_tol=2e-5, g_tol=2e-4):
    names = ("o", "lse", "dq", "dk", "dv")
    for n, a, b in zip(names, got, ref):
        b = b.to(a.dtype)
        tol = o_tol if n in ("o", "lse") else g_tol
        scale = max(1.0, float(b[torch.isfinite(b)].abs().max())) if b.numel() else 1.0
        if n == "lse":
            assert torch.equal(torch.isinf(a), torch.isinf(b)), (what, n)
            a, b = a[torch.isfinite(b)], b[torch.isfinite(b)]
        err = float((a - b).abs().max()) if a.numel() else 0.0
        assert err <= tol * scale, (what, n, err, scale)


def _inputs(B, Sq, Sk, H, D, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    mk = lambda S: torch.randn(B, S, H, D, generator=g).to(DEV)  # noqa: E731
    return mk(Sq), mk(Sk), mk(Sk), mk(Sq)


@pytest.mark.gpu
@pytest.mark.parametrize("D", [32, 64, 128])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("Sq,Sk", [(128, 128), (77, 77), (130, 200), (300, 96)])
def test_f32_kernel_matches_fp64(D, causal, Sq, Sk):
    q, k, v, do = _inputs(2, Sq, Sk, 3, D)
    scale = 1.0 / math.sqrt(D)
    got = _run(q, k, v, do, scale, causal)
    _check(got[:5], _ref(q, k, v, do, scale, causal), (D, causal, Sq, Sk))


@pytest.mark.gpu
def test_f32_kernel_k_lens_and_padding_rows():
    q, k, v, do = _inputs(3, 150, 150, 2, 64, seed=1)
    k_lens = torch.tensor([150, 33, 1], dtype=torch.int32, device=DEV)
    got = _run(q, k, v, do, 0.125, False, k_lens=k_lens)
    ref = _ref(q, k, v, do, 0.125, False, k_lens=k_lens)
    _check(got[:5], ref, "k_lens")
    assert float(got[3][1, 33:].abs().max()) == 0.0 and float(got[4][2, 1:].abs().max()) == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["1h1k", "b1qk", "bhqk"])
@pytest.mark.parametrize("causal", [False, True])
def test_f32_kernel_additive_bias(shape, causal):
    from apex.contrib.multihead_attn.attention import prepare_bias

    B, Sq, Sk, H, D = 2, 96, 160, 4, 64
    q, k, v, do = _inputs(B, Sq, Sk, H, D, seed=2)
    dims = {"1h1k": (1, H, 1, Sk), "b1qk": (B, 1, Sq, Sk), "bhqk": (B, H, Sq, Sk)}[shape]
    g = torch.Generator(device="cpu").manual_seed(3)
    bias = torch.randn(*dims, generator=g).to(DEV)
    bias[..., 5] = float("-inf")  # a masked key column (every row keeps others visible)
    kb = prepare_bias(bias, B, H, Sq, Sk, torch.float32)
    got = _run(q, k, v, do, 0.125, causal, bias=kb)
    _check(got[:5], _ref(q, k, v, do, 0.125, causal, bias=bias), (shape, causal))


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("p", [0.1, 0.5])
def test_f32_kernel_dropout_matches_masked_reference(causal, p):
    B, Sq, Sk, H, D = 2, 100, 170, 3, 64
    q, k, v, do = _inputs(B, Sq, Sk, H, D, seed=4)
    seed, offset = 0x1234_5678_9ABC, 0x0000_0000_0040
    got = _run(q, k, v, do, 0.125, causal, p=p, seed=seed, offset=offset)
    thresh = min(255, max(1, int(p * 256 + 0.5)))
    keep = _keep_from_words(got[5], B, H, Sq, Sk)
    # the stored bits are the shared dropout stream (same as the 16-bit kernels' debug mask);
    # with a causal mask only the blocks a row's query block reaches are drawn
    want = _C().flash_dropout_mask(B, H, Sq, Sk, p, seed, offset, torch.device(DEV)).view(B, H, Sq, Sk)
    if causal:
        q_blk_end = (torch.arange(Sq, device=DEV) // 128 + 1) * 128
        seen = (torch.arange(Sk, device=DEV)[None, :] // 32 * 32) < q_blk_end[:, None]
        assert torch.equal(keep[:, :, seen], want[:, :, seen].to(keep.dtype))
    else:
        assert torch.equal(keep, want.to(keep.dtype))
    ref = _ref(q, k, v, do, 0.125, causal, keep=keep, drop_scale=256.0 / (256 - thresh))
    _check(got[:5], ref, ("dropout", causal, p))


@pytest.mark.gpu
def test_f32_attention_dispatch_uses_kernel_and_is_memory_lean():
    """The public entry (apex.contrib.multihead_attn.attention) takes fp32 device tensors to the
    kernel: no [B, h, S, S] temporaries forward or backward."""
    from apex.contrib.multihead_attn import attention as att

    B, S, H, D = 4, 1024, 8, 64
    q, k, v = (torch.randn(B, S, H, D, device=DEV, requires_grad=True) for _ in range(3))
    assert att._native_ok(q, None)
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    o = att.attention(q, k, v, causal=True)
    o.sum().backward()
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated() - base
    # o, dO and the three gradients are ~8 MB each; one fp32 [B, h, S, S] score tensor is 128 MB
    assert peak < 0.5 * B * H * S * S * 4, peak
    o_ref = att.attention_reference(q.detach(), k.detach(), v.detach(), causal=True)
    torch.testing.assert_close(o.detach(), o_ref, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_f32_kernel_bias_dropout_causal_klens_together():
    """Every option at once: additive bias, dropout, causal mask and per-batch key lengths."""
    from apex.contrib.multihead_attn.attention import prepare_bias

    B, Sq, Sk, H, D = 2, 150, 150, 2, 64
    q, k, v, do = _inputs(B, Sq, Sk, H, D, seed=7)
    g = torch.Generator(device="cpu").manual_seed(8)
    bias = (torch.randn(1, H, Sq, Sk, generator=g) * 0.5).to(DEV)
    k_lens = torch.tensor([150, 97], dtype=torch.int32, device=DEV)
    p, seed, offset = 0.2, 77, 5
    kb = prepare_bias(bias, B, H, Sq, Sk, torch.float32)
    got = _run(q, k, v, do, 0.125, True, p=p, k_lens=k_lens, bias=kb, seed=seed, offset=offset)
    thresh = min(255, max(1, int(p * 256 + 0.5)))
    keep = _keep_from_words(got[5], B, H, Sq, Sk)
    ref = _ref(q, k, v, do, 0.125, True, k_lens=k_lens, bias=bias, keep=keep, drop_scale=256.0 / (256 - thresh))
    _check(got[:5], ref, "all options")
