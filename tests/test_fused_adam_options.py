"""FusedAdam options on the CPU path (the HIP kernel runs the same arithmetic; GPU coverage in
tests/test_optim_mixed_gpu.py): master_weights (fp32 masters of bf16 params inside the
optimizer), the legacy explicit-list step(grads, output_params, scale, grad_norms) with
max_grad_norm clipping, and capturable's GPU-placement check."""
import pytest
import torch

from apex.optimizers import FusedAdam


def _ref_adamw(p32, grads, lr, wd, steps):
    p = p32.clone().requires_grad_(True)
    opt = torch.optim.AdamW([p], lr=lr, weight_decay=wd, eps=1e-8)
    for g in grads:
        p.grad = g.float().clone()
        opt.step()
    return p.detach()


def test_master_weights_bf16_params():
    torch.manual_seed(0)
    w32 = torch.randn(64)
    p = torch.nn.Parameter(w32.to(torch.bfloat16))
    opt = FusedAdam([p], lr=1e-2, weight_decay=0.01, master_weights=True)
    grads = [torch.randn(64).to(torch.bfloat16) for _ in range(5)]
    for g in grads:
        p.grad = g.clone()
        opt.step()
    ref = _ref_adamw(w32.to(torch.bfloat16).float(), grads, 1e-2, 0.01, 5)
    master = opt.state[p]["master_param"]
    assert master.dtype == torch.float32 and p.dtype == torch.bfloat16
    torch.testing.assert_close(master, ref, rtol=1e-5, atol=1e-6)  # fp32 master tracks fp32 Adam
    torch.testing.assert_close(p.data, ref.to(torch.bfloat16))      # model copy = rounded master
    sd = opt.state_dict()
    assert "master_param" in sd["state"][0]


def test_legacy_explicit_lists_and_clipping():
    torch.manual_seed(1)
    master = torch.nn.Parameter(torch.randn(32))
    out16 = torch.zeros(32, dtype=torch.float16)
    opt = FusedAdam([master], lr=1e-2, weight_decay=0.0, max_grad_norm=1.0)
    g = torch.randn(32) * 10.0
    scale = 4.0
    norm = float((g).norm())  # norm of the scaled grads
    ref = master.detach().clone()
    opt.step(grads=[g * 1.0], output_params=[out16], scale=scale, grad_norms=[norm])
    clip = (norm / scale + 1e-6) / 1.0
    ref_p = _ref_adamw(ref, [g / scale / clip], 1e-2, 0.0, 1)
    torch.testing.assert_close(master.detach(), ref_p, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(out16, ref_p.half())


def test_capturable_requires_gpu_params():
    with pytest.raises(RuntimeError, match="capturable"):
        FusedAdam([torch.nn.Parameter(torch.zeros(2))], capturable=True)
