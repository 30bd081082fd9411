"""Numerics of the HIP kernels against plain PyTorch fp32 references (GPU only)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
DTYPES = [torch.float32, torch.float16, torch.bfloat16]
TOL = {torch.float32: 1e-5, torch.float16: 2e-3, torch.bfloat16: 1.6e-2}


def _C():
    import apex._ext as e

    return e.require()


def test_native_extension_loaded_once():
    C = _C()
    assert C.arch == "gfx950"
    maps = open("/proc/self/maps").read()
    hips = {l.split()[-1] for l in maps.splitlines() if "libamdhip64" in l}
    assert len(hips) == 1, hips


def _tensors(sizes, dtype, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return [torch.randn(s, device=DEV, dtype=torch.float32, generator=g).to(dtype) for s in sizes]


SIZES = [1, 7, 8, 1000, 32768, 32769, 100003, 1 << 18]


@pytest.mark.parametrize("din", DTYPES)
@pytest.mark.parametrize("dout", DTYPES)
def test_mt_scale(din, dout):
    from apex.multi_tensor_apply import multi_tensor_applier
    from apex.multi_tensor_apply.ops import multi_tensor_scale

    xs = _tensors(SIZES, din)
    ys = [torch.empty_like(x, dtype=dout) for x in xs]
    flag = torch.zeros(1, dtype=torch.int32, device=DEV)
    multi_tensor_applier(multi_tensor_scale, flag, [xs, ys], 0.125)
    assert int(flag) == 0
    for x, y in zip(xs, ys):
        ref = (x.float() * 0.125).to(dout)
        torch.testing.assert_close(y, ref, rtol=TOL[dout], atol=TOL[dout])
    xs[3][17] = float("inf")
    multi_tensor_applier(multi_tensor_scale, flag, [xs, ys], 0.125)
    assert int(flag) == 1


@pytest.mark.parametrize("dt", DTYPES)
def test_mt_l2norm(dt):
    from apex.multi_tensor_apply import multi_tensor_applier
    from apex.multi_tensor_apply.ops import multi_tensor_l2norm

    xs = _tensors(SIZES, dt, 1)
    flag = torch.zeros(1, dtype=torch.int32, device=DEV)
    tot, per = multi_tensor_applier(multi_tensor_l2norm, flag, [xs], True)
    ref_per = torch.stack([x.double().norm() for x in xs]).float()
    torch.testing.assert_close(per, ref_per, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(tot[0], ref_per.double().pow(2).sum().sqrt().float(), rtol=1e-4, atol=1e-4)
    assert int(flag) == 0


def test_mt_axpby():
    from apex.multi_tensor_apply import multi_tensor_applier
    from apex.multi_tensor_apply.ops import multi_tensor_axpby

    xs = _tensors(SIZES, torch.bfloat16, 2)
    ys = _tensors(SIZES, torch.float32, 3)
    out = [torch.empty_like(y) for y in ys]
    flag = torch.zeros(1, dtype=torch.int32, device=DEV)
    multi_tensor_applier(multi_tensor_axpby, flag, [xs, ys, out], 0.5, -2.0, -1)
    for x, y, o in zip(xs, ys, out):
        torch.testing.assert_close(o, 0.5 * x.float() - 2.0 * y, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("adamw", [True, False])
def test_fused_adam_matches_reference(gdt, adamw):
    from apex.multi_tensor_apply import ops

    sizes = [3, 4096, 70001]
    ps = _tensors(sizes, torch.float32, 4)
    gs = _tensors(sizes, gdt, 5)
    ms = [torch.zeros_like(p) for p in ps]
    vs = [torch.zeros_like(p) for p in ps]
    ps2 = [p.clone().cpu() for p in ps]
    gs2 = [g.clone().cpu() for g in gs]
    ms2 = [m.clone().cpu() for m in ms]
    vs2 = [v.clone().cpu() for v in vs]
    for step in (1, 2, 3):
        ops.multi_tensor_adam(32768, None, [gs, ps, ms, vs], 1e-2, 0.9, 0.999, 1e-8, step,
                              int(adamw), True, 0.01)
        ops.multi_tensor_adam(32768, None, [gs2, ps2, ms2, vs2], 1e-2, 0.9, 0.999, 1e-8, step,
                              int(adamw), True, 0.01)
    for p, p2 in zip(ps, ps2):
        torch.testing.assert_close(p.cpu(), p2, rtol=1e-5, atol=1e-6)


def test_fused_sgd_matches_reference():
    from apex.multi_tensor_apply import ops

    sizes = [5, 8192, 33333]
    ps = _tensors(sizes, torch.float32, 6)
    gs = _tensors(sizes, torch.bfloat16, 7)
    moms = [torch.zeros_like(p) for p in ps]
    cps = [torch.empty_like(p, dtype=torch.bfloat16) for p in ps]
    ps2 = [p.clone().cpu() for p in ps]
    gs2 = [g.clone().cpu() for g in gs]
    moms2 = [m.clone().cpu() for m in moms]
    for first in (True, False, False):
        ops.multi_tensor_sgd(32768, None, [gs, ps, moms, cps], 1e-4, 0.9, 0.0, 0.1, True, first, False, 0.5)
        ops.multi_tensor_sgd(32768, None, [gs2, ps2, moms2], 1e-4, 0.9, 0.0, 0.1, True, first, False, 0.5)
    for p, p2, c in zip(ps, ps2, cps):
        torch.testing.assert_close(p.cpu(), p2, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(c, p.bfloat16(), rtol=0, atol=0)


@pytest.mark.parametrize("nvlamb", [False, True])
def test_fused_lamb_optimizer_matches_reference(nvlamb):
    from apex.optimizers import FusedLAMB

    torch.manual_seed(0)
    shapes = [(64, 33), (128,), (1000, 7)]
    params = [torch.nn.Parameter(torch.randn(s, device=DEV)) for s in shapes]
    ref = [torch.nn.Parameter(p.detach().cpu().clone()) for p in params]
    o1 = FusedLAMB([{"params": params[:2], "weight_decay": 0.01}, {"params": params[2:], "weight_decay": 0.0}],
                   lr=1e-2, max_grad_norm=0.5, use_nvlamb=nvlamb)
    o2 = FusedLAMB([{"params": ref[:2], "weight_decay": 0.01}, {"params": ref[2:], "weight_decay": 0.0}],
                   lr=1e-2, max_grad_norm=0.5, use_nvlamb=nvlamb)
    for it in range(3):
        for p, r in zip(params, ref):
            gg = torch.randn(p.shape) * (it + 1)
            p.grad = gg.to(DEV)
            r.grad = gg.clone()
        o1.step()
        o2.step()
    for p, r in zip(params, ref):
        torch.testing.assert_close(p.detach().cpu(), r.detach(), rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("cols,rows", [(1024, 333), (1600, 333), (768, 333), (64, 333), (100, 333), (4096, 333),
                                       (5000, 333), (2560, 333), (2056, 333), (3072, 333), (2560, 7000)])
@pytest.mark.parametrize("rms", [False, True])
def test_layer_norm_fwd_bwd(dt, cols, rows, rms):
    """cols 2056..4096 run the wide-row backward (ln_bwd_wide), rows 7000 several rows per wave."""
    from apex.normalization import FusedLayerNorm, FusedRMSNorm

    torch.manual_seed(cols)
    x = torch.randn(rows, cols, device=DEV).to(dt).requires_grad_(True)
    mod = (FusedRMSNorm if rms else FusedLayerNorm)(cols).to(DEV).to(dt)
    with torch.no_grad():
        mod.weight.normal_()
        if not rms:
            mod.bias.normal_()
    y = mod(x)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    w = mod.weight.detach().float().requires_grad_(True)
    if rms:
        yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + mod.eps) * w
    else:
        b = mod.bias.detach().float().requires_grad_(True)
        yr = torch.nn.functional.layer_norm(xr, (cols,), w, b, mod.eps)
    yr.backward(dy.float())
    tol = max(TOL[dt], 1e-4)
    torch.testing.assert_close(y.float(), yr, rtol=tol, atol=tol * 4)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=tol * 2, atol=tol * 8)
    torch.testing.assert_close(mod.weight.grad.float(), w.grad, rtol=tol * 4, atol=tol * 40)
    if not rms:
        torch.testing.assert_close(mod.bias.grad.float(), b.grad, rtol=tol * 4, atol=tol * 40)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("V", [30528, 1000, 50257])
@pytest.mark.parametrize("smoothing", [0.0, 0.1])
def test_xentropy(dt, V, smoothing):
    from apex.contrib.xentropy import SoftmaxCrossEntropyLoss

    torch.manual_seed(V)
    N = 77
    x = (torch.randn(N, V, device=DEV) * 3).to(dt).requires_grad_(True)
    y = torch.randint(0, V, (N,), device=DEV)
    y[5] = 0  # padding row
    loss = SoftmaxCrossEntropyLoss.apply(x, y, smoothing, 0, False)
    g = torch.rand(N, device=DEV)
    loss.backward(g)
    xr = x.detach().float().requires_grad_(True)
    lse = torch.logsumexp(xr, -1)
    lr = (1 - smoothing) * (lse - xr.gather(1, y[:, None]).squeeze(1)) + smoothing * (lse - xr.mean(-1))
    lr = torch.where(y != 0, lr, torch.zeros_like(lr))
    lr.backward(g)
    torch.testing.assert_close(loss, lr, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=TOL[dt] * 2, atol=TOL[dt])


def test_update_scale_device():
    from apex.multi_tensor_apply.ops import update_scale_

    s = torch.full((), 1024.0, device=DEV)
    tr = torch.zeros(1, dtype=torch.int32, device=DEV)
    of = torch.ones(1, dtype=torch.int32, device=DEV)
    update_scale_(s, tr, of, 2.0, 0.5, 3)
    assert float(s) == 512.0
    of.zero_()
    for _ in range(3):
        update_scale_(s, tr, of, 2.0, 0.5, 3)
    assert float(s) == 1024.0 and int(tr) == 0
