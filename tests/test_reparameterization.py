"""apex.reparameterization (R-20..22) + Fused_Weight_Norm (K-03): CPU reference path and GPU kernels."""
import pytest
import torch
from torch import nn

from apex.fp16_utils import Fused_Weight_Norm
from apex.reparameterization import apply_weight_norm, remove_weight_norm


@pytest.mark.parametrize("dim", [0, 1, None])
def test_weight_norm_linear_matches_torch(dim):
    torch.manual_seed(0)
    m = nn.Linear(20, 40)
    ref = nn.Linear(20, 40)
    ref.load_state_dict(m.state_dict())
    apply_weight_norm(m, "weight", dim=dim)
    assert hasattr(m, "weight_g") and hasattr(m, "weight_v")
    ref = torch.nn.utils.parametrizations.weight_norm(ref, "weight", dim=dim)
    x = torch.randn(8, 20)
    y, yr = m(x), ref(x)
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-6)
    y.sum().backward()
    yr.sum().backward()
    torch.testing.assert_close(m.weight_v.grad, ref.parametrizations.weight.original1.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(m.weight_g.grad.reshape(-1),
                               ref.parametrizations.weight.original0.grad.reshape(-1), rtol=1e-4, atol=1e-6)


def test_weight_recomputed_after_update_and_remove():
    torch.manual_seed(1)
    m = apply_weight_norm(nn.Linear(5, 7), "weight")
    x = torch.randn(3, 5)
    y1 = m(x)
    with torch.no_grad():
        m.weight_g.mul_(2.0)
        y2 = m(x)
    torch.testing.assert_close(y2 - m.bias, 2 * (y1 - m.bias).detach(), rtol=1e-5, atol=1e-6)
    remove_weight_norm(m, "weight")
    assert isinstance(m.weight, nn.Parameter) and not hasattr(m, "weight_g")
    torch.testing.assert_close(m(x), y2, rtol=1e-5, atol=1e-6)


def test_apply_all_skips_vectors():
    m = nn.Sequential(nn.Linear(4, 4), nn.Conv2d(3, 6, 3))
    apply_weight_norm(m)
    names = {n for n, _ in m.named_parameters()}
    assert "0.weight_g" in names and "1.weight_v" in names and "0.bias" in names


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape,dim", [((64, 33), 0), ((48, 8, 3, 3), 0), ((40, 70), 1), ((5, 6, 129), 2)])
def test_fused_weight_norm_kernel(dt, shape, dim):
    torch.manual_seed(2)
    v = torch.randn(shape, device="cuda").to(dt).requires_grad_(True)
    gshape = [1] * len(shape)
    gshape[dim] = shape[dim]
    g = (torch.rand(gshape, device="cuda") + 0.5).to(dt).requires_grad_(True)
    w = Fused_Weight_Norm.apply(v, g, dim)
    dw = torch.randn_like(w)
    w.backward(dw)
    vr, gr = v.detach().double().requires_grad_(True), g.detach().double().requires_grad_(True)
    dims = [d for d in range(len(shape)) if d != dim]
    wr = gr * vr / vr.pow(2).sum(dims, keepdim=True).sqrt()
    wr.backward(dw.double())
    tol = {torch.float32: 1e-5, torch.bfloat16: 2e-2, torch.float16: 3e-3}[dt]
    torch.testing.assert_close(w.double(), wr, rtol=tol, atol=tol)
    torch.testing.assert_close(v.grad.double(), vr.grad, rtol=tol * 4, atol=tol * 4)
    torch.testing.assert_close(g.grad.double(), gr.grad, rtol=tol * 4, atol=tol * 4)
