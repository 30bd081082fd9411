"""SyncBatchNorm (NS-04): multi-process gloo equivalence with single-process BatchNorm over the
full batch (CPU reference path), plus GPU kernel numerics (marker gpu)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from torch import nn


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, sizes, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.set_num_threads(1)
        from apex.parallel import SyncBatchNorm, convert_syncbn_model

        torch.manual_seed(0)
        C = 6
        xs = [torch.randn(n, C, 5, 4) * 3 + 1 for n in sizes]  # uneven per-rank batches
        full = torch.cat(xs).requires_grad_(True)
        ref = nn.BatchNorm2d(C)
        with torch.no_grad():
            ref.weight.uniform_(0.5, 1.5)
            ref.bias.uniform_(-0.5, 0.5)
        sbn = convert_syncbn_model(nn.Sequential(nn.BatchNorm2d(C)))[0]
        assert isinstance(sbn, SyncBatchNorm)
        sbn.load_state_dict(ref.state_dict())
        yr = ref(full)
        g = torch.randn_like(yr)
        yr.backward(g)
        off = sum(sizes[:rank])
        x = xs[rank].clone().requires_grad_(True)
        y = sbn(x)
        y.backward(g[off:off + sizes[rank]])
        torch.testing.assert_close(y, yr[off:off + sizes[rank]], rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(x.grad, full.grad[off:off + sizes[rank]], rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(sbn.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(sbn.bias.grad, ref.bias.grad, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(sbn.running_mean, ref.running_mean, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(sbn.running_var, ref.running_var, rtol=1e-5, atol=1e-6)
        sbn.eval()
        ref.eval()
        torch.testing.assert_close(sbn(xs[rank]), ref(xs[rank]), rtol=1e-5, atol=1e-5)
        q.put((rank, "ok"))
    except Exception:
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_syncbn_matches_full_batch_bn():
    sizes = [3, 5]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, sizes, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert all(r[1] == "ok" for r in res), res


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape,channel_last", [((8, 16, 7, 7), False), ((4, 64, 20, 9), False),
                                                ((6, 5, 3, 32), True), ((33, 12), False),
                                                # vectorised paths: NCHW planes % 8, NHWC channels % 8
                                                ((4, 64, 16, 8), False), ((2, 32, 56, 56), False),
                                                ((4, 7, 9, 64), True), ((8, 14, 14, 256), True),
                                                ((2, 7, 7, 2048), True), ((3, 24), False)])
def test_syncbn_kernels_single_process(dt, shape, channel_last):
    from apex.parallel import SyncBatchNorm

    torch.manual_seed(1)
    C = shape[-1] if channel_last else shape[1]
    x = (torch.randn(shape, device="cuda") * 2 + 0.5).to(dt).requires_grad_(True)
    m = SyncBatchNorm(C, channel_last=channel_last).cuda()
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5)
        m.bias.uniform_(-0.5, 0.5)
    y = m(x)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    xin = xr.movedim(-1, 1) if channel_last else xr
    ref = nn.BatchNorm2d(C).cuda() if xin.dim() == 4 else nn.BatchNorm1d(C).cuda()
    ref.load_state_dict({k: v for k, v in m.state_dict().items() if k != "num_batches_tracked"}, strict=False)
    with torch.no_grad():
        ref.running_mean.zero_()
        ref.running_var.fill_(1)
    yr = ref(xin)
    yr = yr.movedim(1, -1) if channel_last else yr
    yr.backward(dy.float())
    tol = {torch.float32: 1e-4, torch.bfloat16: 3e-2, torch.float16: 5e-3}[dt]
    torch.testing.assert_close(y.float(), yr, rtol=tol, atol=tol)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=tol * 2, atol=tol * 2)
    torch.testing.assert_close(m.weight.grad.float(), ref.weight.grad, rtol=tol * 4, atol=tol * 20)
    torch.testing.assert_close(m.running_mean, ref.running_mean, rtol=1e-3, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_syncbn_channels_last_memory_format_and_large_mean(dt):
    """A torch channels_last NCHW tensor takes the NHWC kernels on the zero-copy view; inputs with
    a mean far from zero check the Welford partial merges (a sum / sum-of-squares reduction would
    lose the variance to cancellation at mean 100, std 1)."""
    from apex.parallel import SyncBatchNorm

    torch.manual_seed(2)
    N, C, H, W = 16, 128, 28, 28
    x = (torch.randn(N, C, H, W, device="cuda") + 100.0).to(dt).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    m = SyncBatchNorm(C).cuda()
    y = m(x)
    dy = torch.randn_like(y)
    y.backward(dy)
    # fp64 reference: an fp32 library BatchNorm itself loses ~1e-3 at mean 100
    xr = x.detach().double().requires_grad_(True)
    ref = nn.BatchNorm2d(C).cuda().double()
    yr = ref(xr)
    yr.backward(dy.double())
    tol = 3e-2 if dt == torch.bfloat16 else 1e-3
    torch.testing.assert_close(y.float(), yr.float(), rtol=tol, atol=tol)
    torch.testing.assert_close(x.grad.float(), xr.grad.float(), rtol=2 * tol, atol=2 * tol)
    torch.testing.assert_close(m.running_var, ref.running_var.float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("channels_last", [False, True])
def test_syncbn_fused_residual_relu_cpu(channels_last):
    """relu(BN(x) + z) through SyncBatchNorm(fuse_relu=True)(x, z): output and gradients of x, z,
    weight, bias against the separate-op composition (CPU reference path)."""
    from apex.parallel import SyncBatchNorm

    torch.manual_seed(3)
    x = torch.randn(4, 16, 5, 6, dtype=torch.float32)
    z = torch.randn(4, 16, 5, 6, dtype=torch.float32)
    if channels_last:
        x, z = x.to(memory_format=torch.channels_last), z.to(memory_format=torch.channels_last)
    bn = SyncBatchNorm(16, fuse_relu=True)
    ref = torch.nn.BatchNorm2d(16)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        ref.weight.copy_(bn.weight)
        ref.bias.copy_(bn.bias)
    x1, z1, x2, z2 = (t.clone().requires_grad_() for t in (x, z, x, z))
    y = bn(x1, z1)
    yr = torch.relu(ref(x2) + z2)
    dy = torch.randn_like(yr)
    y.backward(dy)
    yr.backward(dy)
    torch.testing.assert_close(y, yr, atol=1e-5, rtol=1e-4)  # the reference path computes in fp32
    for a, b in ((x1.grad, x2.grad), (z1.grad, z2.grad), (bn.weight.grad, ref.weight.grad),
                 (bn.bias.grad, ref.bias.grad)):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(bn.running_mean, ref.running_mean)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape,mem", [((8, 64, 14, 14), "cl"), ((4, 32, 16, 8), "nchw"), ((6, 5, 7, 7), "nchw"),
                                       ((4, 24, 9, 9), "cl")])
@pytest.mark.parametrize("with_z", [True, False])
def test_syncbn_fused_residual_relu_gpu(dt, shape, mem, with_z):
    """relu(BN(x) + z) in the HIP kernels (vectorised NHWC / NCHW and the scalar fallback for odd
    channel / plane counts): output and the x, z, weight, bias gradients vs the fp32 composition."""
    from apex.parallel import SyncBatchNorm

    torch.manual_seed(4)
    C = shape[1]
    fmt = torch.channels_last if mem == "cl" else torch.contiguous_format
    x = (torch.randn(shape, device="cuda") * 2 + 0.3).to(dt).contiguous(memory_format=fmt).requires_grad_(True)
    z = torch.randn(shape, device="cuda").to(dt).contiguous(memory_format=fmt).requires_grad_(True)
    m = SyncBatchNorm(C, fuse_relu=True).cuda()
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5)
        m.bias.uniform_(-0.5, 0.5)
    y = m(x, z) if with_z else m(x)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, zr = (t.detach().float().requires_grad_(True) for t in (x, z))
    ref = nn.BatchNorm2d(C).cuda()
    ref.load_state_dict({k: v for k, v in m.state_dict().items() if k != "num_batches_tracked"}, strict=False)
    with torch.no_grad():
        ref.running_mean.zero_()
        ref.running_var.fill_(1)
    yr = torch.relu(ref(xr) + zr) if with_z else torch.relu(ref(xr))
    yr.backward(dy.float())
    tol = 3e-2 if dt == torch.bfloat16 else 1e-4
    torch.testing.assert_close(y.float(), yr, rtol=tol, atol=tol)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2 * tol, atol=2 * tol)
    if with_z:
        torch.testing.assert_close(z.grad.float(), zr.grad, rtol=tol, atol=tol)
    torch.testing.assert_close(m.weight.grad.float(), ref.weight.grad, rtol=tol * 4, atol=tol * 20)
    torch.testing.assert_close(m.bias.grad.float(), ref.bias.grad, rtol=tol * 4, atol=tol * 20)


def _running_stats_case(device, dt, momentum, channel_last_mem):
    from apex.parallel import SyncBatchNorm

    torch.manual_seed(5)
    C = 24
    m = SyncBatchNorm(C, momentum=momentum).to(device)
    ref = nn.BatchNorm2d(C, momentum=momentum).to(device)
    fmt = torch.channels_last if channel_last_mem else torch.contiguous_format
    for step in range(3):
        x = (torch.randn(6, C, 5, 7, device=device) * (step + 1) + step).to(dt).contiguous(memory_format=fmt)
        m(x)
        ref(x.float())
    assert int(m.num_batches_tracked) == 3
    torch.testing.assert_close(m.running_mean, ref.running_mean, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(m.running_var, ref.running_var, rtol=1e-3, atol=1e-3)
    m.eval()
    ref.eval()
    x = torch.randn(2, C, 5, 7, device=device).to(dt)
    tol = 3e-2 if dt == torch.bfloat16 else 1e-4
    torch.testing.assert_close(m(x).float(), ref(x.float()), rtol=tol, atol=tol)


@pytest.mark.parametrize("momentum", [0.1, None])
def test_syncbn_running_stats_cpu(momentum):
    """Running mean / unbiased running variance / num_batches_tracked over several steps vs
    torch BatchNorm, incl. momentum=None (cumulative average)."""
    _running_stats_case("cpu", torch.float32, momentum, False)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("momentum", [0.1, None])
@pytest.mark.parametrize("cl", [False, True])
def test_syncbn_running_stats_gpu(dt, momentum, cl):
    """The fused combine kernel (invstd + in-place fp32 running-statistics update +
    num_batches_tracked in the same launch) against torch BatchNorm over several steps."""
    _running_stats_case("cuda", dt, momentum, cl)
