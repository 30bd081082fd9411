"""Query-blocked memory-efficient attention (apex.contrib.multihead_attn.chunked) against the
fp32 reference composition on CPU: outputs and q/k/v gradients, causal / key-length masks, and the
gradient of a TRAINABLE additive bias (ALiBi-style [1, h, Sq, Sk] and per-head [h, 1, Sk]
broadcasts). The GPU run at S = 2048 in fp32 is tests/test_attention_fp32_gpu.py."""
import pytest
import torch

from apex.contrib.multihead_attn.attention import attention_reference
from apex.contrib.multihead_attn.chunked import chunked_attention


def _inputs(B=2, S=40, H=3, d=16, seed=0):
    g = torch.Generator().manual_seed(seed)
    q, k, v = (torch.randn(B, S, H, d, generator=g, dtype=torch.float64) for _ in range(3))
    return q, k, v


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("bias_kind", [None, "alibi", "perhead"])
def test_chunked_matches_reference(causal, bias_kind):
    q, k, v = _inputs()
    B, S, H, d = q.shape
    bias = None
    if bias_kind == "alibi":
        slopes = torch.tensor([0.5, 0.25, 0.125], dtype=torch.float64)
        pos = torch.arange(S, dtype=torch.float64)
        bias = (-(pos[None, :] - pos[:, None]).abs())[None, None] * slopes[None, :, None, None]
        bias = bias.clone().requires_grad_(True)  # [1, H, S, S]
    elif bias_kind == "perhead":
        bias = torch.randn(H, 1, S, dtype=torch.float64).requires_grad_(True)
    k_lens = torch.tensor([S, S - 7])
    outs, grads = [], []
    for fn in (attention_reference, lambda *a, **kw: chunked_attention(*a, **kw, block=16)):
        qq, kk, vv = (t.clone().requires_grad_(True) for t in (q, k, v))
        bb = bias.detach().clone().requires_grad_(True) if bias is not None else None
        o = fn(qq, kk, vv, bb, 0.0, causal, None, k_lens)
        (o * torch.linspace(-1, 1, o.numel(), dtype=o.dtype).view_as(o)).sum().backward()
        outs.append(o)
        grads.append([qq.grad, kk.grad, vv.grad] + ([bb.grad] if bb is not None else []))
    torch.testing.assert_close(outs[1], outs[0], rtol=1e-5, atol=2e-6)  # both compute in fp32
    for a, b in zip(grads[1], grads[0]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


def test_chunked_dropout_is_seeded_and_unbiased():
    q, k, v = _inputs(B=1, S=64, H=2, d=8)
    torch.manual_seed(3)
    a = chunked_attention(q, k, v, dropout_p=0.3)
    torch.manual_seed(3)
    b = chunked_attention(q, k, v, dropout_p=0.3)
    torch.testing.assert_close(a, b)
    ref = chunked_attention(q, k, v)
    m = torch.stack([chunked_attention(q, k, v, dropout_p=0.3) for _ in range(200)]).mean(0)
    assert float((m - ref).abs().mean()) < 0.05 * float(ref.abs().mean())
