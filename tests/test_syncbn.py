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
