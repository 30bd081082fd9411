"""apex.contrib.multihead_attn modules vs a plain PyTorch formulation (CPU + GPU)."""
import math

import pytest
import torch
import torch.nn.functional as F

from apex.contrib.multihead_attn import EncdecMultiheadAttn, SelfMultiheadAttn

CASES = [("cpu", torch.float32)]
if torch.cuda.is_available():
    CASES += [pytest.param(("cuda", torch.bfloat16), marks=pytest.mark.gpu)]


def _ref_attn(q, k, v, H, k_lens=None):
    S, B, E = q.shape
    D = E // H
    qh, kh, vh = (t.reshape(t.shape[0], B, H, D).permute(1, 2, 0, 3).float() for t in (q, k, v))
    s = qh @ kh.transpose(-1, -2) / math.sqrt(D)
    if k_lens is not None:
        m = torch.arange(k.shape[0], device=q.device)[None] >= k_lens[:, None]
        s = s.masked_fill(m[:, None, None, :], float("-inf"))
    o = torch.softmax(s, -1) @ vh
    return o.permute(2, 0, 1, 3).reshape(S, B, E)


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("norm_add", [False, True])
def test_self_attn(case, norm_add):
    dev, dt = case
    torch.manual_seed(0)
    S, B, E, H = 24, 3, 128, 2
    m = SelfMultiheadAttn(E, H, dropout=0.0, bias=True, include_norm_add=norm_add).to(dev).to(dt)
    x = torch.randn(S, B, E, device=dev).to(dt)
    kpm = torch.zeros(B, S, dtype=torch.bool, device=dev)
    kpm[1, 20:] = True
    y, _ = m(x, x, x, key_padding_mask=kpm)
    xin = F.layer_norm(x.float(), (E,), m.lyr_nrm.weight.float(), m.lyr_nrm.bias.float()) if norm_add else x.float()
    qkv = F.linear(xin, m.in_proj_weight.float(), m.in_proj_bias.float())
    q, k, v = qkv.chunk(3, -1)
    ctx = _ref_attn(q, k, v, H, (~kpm).sum(1))
    yr = F.linear(ctx, m.out_proj_weight.float(), m.out_proj_bias.float())
    if norm_add:
        yr = yr + x.float()
    tol = 1e-4 if dt == torch.float32 else 5e-2
    torch.testing.assert_close(y.float(), yr, rtol=tol, atol=tol)


@pytest.mark.parametrize("case", CASES)
def test_encdec_attn(case):
    dev, dt = case
    torch.manual_seed(1)
    Sq, Sk, B, E, H = 10, 17, 2, 128, 2
    m = EncdecMultiheadAttn(E, H, bias=True).to(dev).to(dt)
    q = torch.randn(Sq, B, E, device=dev).to(dt)
    kk = torch.randn(Sk, B, E, device=dev).to(dt)
    y, _ = m(q, kk, kk)
    qq = F.linear(q.float(), m.in_proj_weight_q.float(), m.in_proj_bias_q.float())
    kv = F.linear(kk.float(), m.in_proj_weight_kv.float(), m.in_proj_bias_kv.float())
    k, v = kv.view(Sk, B, 2, E).unbind(2)
    yr = F.linear(_ref_attn(qq, k, v, H), m.out_proj_weight.float(), m.out_proj_bias.float())
    tol = 1e-4 if dt == torch.float32 else 5e-2
    torch.testing.assert_close(y.float(), yr, rtol=tol, atol=tol)
