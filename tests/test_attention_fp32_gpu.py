"""Device attention paths the flash kernels do not take, against the fp32 reference composition:
fp32 inputs at S = 2048 (query-blocked, O(S * block) memory, exact f32 MFMA GEMMs) and a
TRAINABLE ALiBi-style bias with bf16 inputs (its gradient is the blocked score gradient). Both go
through apex.contrib.multihead_attn.attention, i.e. the same dispatch the models use."""
import math

import pytest
import torch

from apex.contrib.multihead_attn.attention import attention, attention_reference


def _loss_grads(fn, q, k, v, bias, causal):
    qq, kk, vv = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    bb = bias.detach().clone().requires_grad_(True) if bias is not None else None
    o = fn(qq, kk, vv, bb, 0.0, causal)
    w = torch.linspace(-1, 1, o.numel(), device=o.device, dtype=torch.float32).view_as(o)
    (o.float() * w).sum().backward()
    return o, [qq.grad, kk.grad, vv.grad] + ([bb.grad] if bb is not None else [])


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
def test_fp32_attention_s2048(causal):
    torch.manual_seed(0)
    B, S, H, d = 2, 2048, 4, 64
    q, k, v = (torch.randn(B, S, H, d, device="cuda") for _ in range(3))
    # warm-up call first: the BLAS library's one-time workspace allocations (first GEMM of a
    # process) are not the attention's memory
    _loss_grads(attention, q, k, v, None, causal)
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    o, g = _loss_grads(attention, q, k, v, None, causal)
    peak = torch.cuda.max_memory_allocated() - base
    o_ref, g_ref = _loss_grads(attention_reference, q, k, v, None, causal)
    torch.testing.assert_close(o, o_ref, rtol=1e-4, atol=1e-5)
    for a, b in zip(g, g_ref):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-4)
    # never the [B, h, S, S] composition: one fp32 score tensor alone would be 128 MB here
    assert peak < 1.5 * B * H * S * S * 4, peak


@pytest.mark.gpu
def test_trainable_alibi_bias_bf16():
    torch.manual_seed(1)
    B, S, H, d = 2, 512, 8, 64
    q, k, v = (torch.randn(B, S, H, d, device="cuda").bfloat16() for _ in range(3))
    slopes = torch.tensor([2.0 ** (-8 * (i + 1) / H) for i in range(H)], device="cuda")
    pos = torch.arange(S, device="cuda", dtype=torch.float32)
    alibi = (-(pos[None, :] - pos[:, None]).abs())[None, None] * slopes[None, :, None, None]  # [1, H, S, S]
    o, g = _loss_grads(attention, q, k, v, alibi, True)
    qf, kf, vf = (t.float() for t in (q, k, v))
    o_ref, g_ref = _loss_grads(attention_reference, qf, kf, vf, alibi, True)
    torch.testing.assert_close(o.float(), o_ref, rtol=2e-2, atol=2e-2)
    for a, b in zip(g, g_ref):
        torch.testing.assert_close(a.float(), b, rtol=3e-2, atol=3e-2)
    assert g[3].shape == alibi.shape and float(g[3].abs().sum()) > 0
