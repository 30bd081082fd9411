"""Flash-attention HIP kernels vs a plain PyTorch fp32 reference (GPU only)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(q, k, v, causal, scale, mask=None, p=0.0, k_lens=None):
    # q,k,v [B,S,H,D] -> fp32 reference
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    Sq, Sk = s.shape[-2], s.shape[-1]
    if causal:
        cm = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(cm, float("-inf"))
    if k_lens is not None:
        km = torch.arange(Sk, device=q.device)[None, :] >= k_lens[:, None].long()
        s = s.masked_fill(km[:, None, None, :], float("-inf"))
    pm = torch.softmax(s, -1)
    pm = torch.nan_to_num(pm)
    if mask is not None:
        pm = pm * mask.float() / (1.0 - p)
    o = torch.matmul(pm, vf)
    return o.transpose(1, 2)


CASES = [
    # B, S, H, D, causal
    (2, 128, 4, 64, False),
    (3, 100, 2, 64, False),
    (2, 257, 3, 64, True),
    (1, 128, 2, 128, False),
    (2, 190, 2, 128, True),
    (1, 512, 2, 64, False),
]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,S,H,D,causal", CASES)
def test_flash_fwd_bwd(dt, B, S, H, D, causal):
    from apex.contrib.multihead_attn.flash import flash_attention_packed

    torch.manual_seed(S * D + int(causal))
    qkv = (torch.randn(B, S, 3, H, D, device=DEV) * 0.8).to(dt).requires_grad_(True)
    scale = 1.0 / math.sqrt(D)
    o = flash_attention_packed(qkv, 0.0, causal, scale)
    do = torch.randn_like(o)
    o.backward(do)
    q, k, v = qkv.detach().float().unbind(2)
    qr, kr, vr = (t.clone().requires_grad_(True) for t in (q, k, v))
    orf = _ref(qr, kr, vr, causal, scale)
    orf.backward(do.float())
    tol = 2e-2 if dt == torch.bfloat16 else 4e-3
    torch.testing.assert_close(o.float(), orf, rtol=tol, atol=tol)
    dq, dk, dv = qkv.grad.float().unbind(2)
    gtol = 5e-2 if dt == torch.bfloat16 else 1e-2
    torch.testing.assert_close(dv, vr.grad, rtol=gtol, atol=gtol)
    torch.testing.assert_close(dk, kr.grad, rtol=gtol, atol=gtol)
    torch.testing.assert_close(dq, qr.grad, rtol=gtol, atol=gtol)


def test_flash_key_lengths():
    from apex.contrib.multihead_attn.flash import flash_attention

    torch.manual_seed(0)
    B, S, H, D = 3, 160, 2, 64
    q, k, v = (torch.randn(B, S, H, D, device=DEV).bfloat16().requires_grad_(True) for _ in range(3))
    kl = torch.tensor([160, 77, 1], dtype=torch.int32, device=DEV)
    o = flash_attention(q, k, v, 0.0, False, None, kl)
    do = torch.randn_like(o)
    o.backward(do)
    refs = [t.detach().float().requires_grad_(True) for t in (q, k, v)]
    orf = _ref(*refs, False, 1 / math.sqrt(D), k_lens=kl)
    orf.backward(do.float())
    torch.testing.assert_close(o.float(), orf, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(k.grad.float(), refs[1].grad, rtol=5e-2, atol=5e-2)
    torch.testing.assert_close(q.grad.float(), refs[0].grad, rtol=5e-2, atol=5e-2)


@pytest.mark.parametrize("causal", [False, True])
def test_flash_dropout_matches_masked_reference(causal):
    import apex._ext as e
    from apex.contrib.multihead_attn import flash

    C = e.require()
    torch.manual_seed(3)
    B, S, H, D, p = 2, 136, 2, 64, 0.1
    qkv = (torch.randn(B, S, 3, H, D, device=DEV) * 0.7).bfloat16().requires_grad_(True)
    torch.manual_seed(11)
    o = flash.flash_attention_packed(qkv, p, causal, None)
    torch.manual_seed(11)
    seed, offset = flash._seed_pair(p, qkv.device)
    mask = C.flash_dropout_mask(B, H, S, S, p, seed, offset, qkv.device)
    keep = mask.float().mean().item()
    assert abs(keep - (1 - p)) < 0.01
    do = torch.randn_like(o)
    o.backward(do)
    q, k, v = (t.float().clone().requires_grad_(True) for t in qkv.detach().unbind(2))
    pq = round(p * 256) / 256  # attention dropout uses 8-bit uniforms
    orf = _ref(q, k, v, causal, 1 / math.sqrt(D), mask=mask, p=pq)
    orf.backward(do.float())
    torch.testing.assert_close(o.float(), orf, rtol=2e-2, atol=2e-2)
    dq, dk, dv = qkv.grad.float().unbind(2)
    torch.testing.assert_close(dv, v.grad, rtol=5e-2, atol=5e-2)
    torch.testing.assert_close(dk, k.grad, rtol=5e-2, atol=5e-2)
    torch.testing.assert_close(dq, q.grad, rtol=5e-2, atol=5e-2)


@pytest.mark.parametrize("S,causal", [(128, False), (200, False), (256, True)])
def test_attention_bwd_bias_colsums(S, causal):
    """flash_attn_bwd's optional dsum output = per-sequence column sums of dq, dk, dv."""
    import apex._ext as e

    C = e.require()
    torch.manual_seed(S)
    B, H, D = 3, 4, 64
    qkv = torch.randn(B, S, 3, H, D, device="cuda").bfloat16()
    q, k, v = qkv.unbind(2)
    scale = D ** -0.5
    o, lse, dmask = C.flash_attn_fwd(q, k, v, causal, scale, 0.0, 0, 0, None)
    do = torch.randn_like(o)
    dqkv = torch.empty_like(qkv)
    dq, dk, dv = dqkv.unbind(2)
    dsum = torch.zeros(B, 3 * H * D, device="cuda")
    C.flash_attn_bwd(do, q, k, v, o, lse, dq, dk, dv, causal, scale, 0.0, 0, 0, None, dmask, dsum)
    ref = dqkv.float().sum(1).reshape(B, 3 * H * D)
    torch.testing.assert_close(dsum, ref, rtol=2e-3, atol=2e-2)
    db = C.partial_colsum(dsum, torch.float32)
    torch.testing.assert_close(db, ref.sum(0), rtol=2e-3, atol=5e-2)
