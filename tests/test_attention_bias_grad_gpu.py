"""Trainable additive attention bias through the flash kernels: the backward kernels write dS into
an fp32 tensor of the bias's broadcast shape (atomically over broadcast dims). Checked against
autograd through the fp32 reference composition, for bf16 (single-kernel backward at Sk <= 128,
two-kernel beyond) and fp32 inputs (csrc/attention_f32.hip), every broadcast layout, causal or
not, and through both public entries (separate q/k/v and the packed QKV projection)."""
import math

import pytest
import torch

from apex.contrib.multihead_attn import attention as att

DEV = "cuda"


def _run(fn, q, k, v, bias, causal, packed):
    qq, kk, vv = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    bb = bias.detach().clone().requires_grad_(True)
    if packed:
        qkv = torch.stack([qq, kk, vv], dim=2)
        o = att.attention_packed(qkv, bb, 0.0, causal)
    else:
        o = fn(qq, kk, vv, bb, 0.0, causal)
    w = torch.linspace(-1, 1, o.numel(), device=o.device, dtype=torch.float32).view_as(o)
    (o.float() * w).sum().backward()
    return o, bb.grad, [qq.grad, kk.grad, vv.grad]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("S", [96, 200])
@pytest.mark.parametrize("shape", ["1hqk", "b1qk", "bhqk", "111k"])
@pytest.mark.parametrize("causal", [False, True])
def test_bias_gradient_matches_reference(dtype, S, shape, causal):
    torch.manual_seed(0)
    B, H, D = 2, 4, 64
    q, k, v = (torch.randn(B, S, H, D, device=DEV).to(dtype) for _ in range(3))
    dims = {"1hqk": (1, H, S, S), "b1qk": (B, 1, S, S), "bhqk": (B, H, S, S), "111k": (1, 1, 1, S)}[shape]
    bias = torch.randn(*dims, device=DEV) * 0.5
    assert att._native_ok(q, bias.requires_grad_(True))
    o, db, g = _run(att.attention, q, k, v, bias, causal, packed=False)
    qf, kf, vf = (t.float() for t in (q, k, v))
    o_ref, db_ref, g_ref = _run(att.attention_reference, qf, kf, vf, bias, causal, packed=False)
    tol = dict(rtol=2e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(o.float(), o_ref, **tol)
    assert db.shape == bias.shape and db.dtype == bias.dtype
    scale = float(db_ref.abs().max())
    err = float((db.float() - db_ref).abs().max())
    assert err <= (2e-2 if dtype == torch.bfloat16 else 1e-4) * max(scale, 1.0), (err, scale)
    for a, b in zip(g, g_ref):
        torch.testing.assert_close(a.float(), b, **(dict(rtol=3e-2, atol=3e-2) if dtype == torch.bfloat16 else tol))


@pytest.mark.gpu
def test_bias_gradient_packed_qkv_bf16():
    torch.manual_seed(1)
    B, S, H, D = 2, 128, 4, 64
    q, k, v = (torch.randn(B, S, H, D, device=DEV).bfloat16() for _ in range(3))
    slopes = torch.tensor([2.0 ** (-8 * (i + 1) / H) for i in range(H)], device=DEV)
    pos = torch.arange(S, device=DEV, dtype=torch.float32)
    alibi = (-(pos[None, :] - pos[:, None]).abs())[None, None] * slopes[None, :, None, None]
    _, db, _ = _run(None, q, k, v, alibi, True, packed=True)
    _, db_ref, _ = _run(att.attention_reference, q.float(), k.float(), v.float(), alibi, True, packed=False)
    err = float((db.float() - db_ref).abs().max())
    assert err <= 2e-2 * max(float(db_ref.abs().max()), 1.0), err
