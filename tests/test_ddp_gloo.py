"""apex.parallel DDP / Reducer correctness on CPU with gloo, world_size 2 and 3.

Generalises the reference race test (tests/distributed/ddp_race_condition_test.py:28-61:
out = (x*a)*b, message_size=1 -> one bucket per param, exact closed-form grad sums)
to any world size, and checks DDP training equals single-process full-batch training.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)


class _Model(torch.nn.Module):
    def __init__(self, n):
        super().__init__()
        self.a = torch.nn.Parameter(torch.ones(n))
        self.b = torch.nn.Parameter(torch.full((n,), 2.0))

    def forward(self, x):
        return (x * self.a) * self.b


def _race_worker(rank, world, port, delay, n, q):
    try:
        _init(rank, world, port)
        from apex.parallel import DistributedDataParallel as DDP

        model = DDP(_Model(n), message_size=1, delay_allreduce=delay)
        x = torch.empty(n)
        for i in range(6):
            model.zero_grad(set_to_none=(i % 2 == 0))
            x.fill_(float(i + rank))
            model(x).sum().backward()
            # grad_a = x*b averaged: 2*mean_r(i+r) ; grad_b = x*a averaged: mean_r(i+r)
            mean_x = i + (world - 1) / 2.0
            ga = model.module.a.grad
            gb = model.module.b.grad
            assert torch.all(ga == 2 * mean_x), (i, ga[:3])
            assert torch.all(gb == mean_x), (i, gb[:3])
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("delay", [False, True])
def test_ddp_race_closed_form(world, delay):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_race_worker, args=(r, world, port, delay, 4096, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] == "ok" for r in res), res


def _equiv_worker(rank, world, port, q):
    try:
        _init(rank, world, port)
        from apex.parallel import DistributedDataParallel as DDP
        from apex.parallel import Reducer

        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
        ref = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
        ref.load_state_dict(net.state_dict())
        if rank == 1:  # DDP must broadcast rank 0's params
            with torch.no_grad():
                for p in net.parameters():
                    p.add_(1.0)
        model = DDP(net, message_size=200)
        opt = torch.optim.SGD(model.parameters(), lr=0.1)
        ropt = torch.optim.SGD(ref.parameters(), lr=0.1)
        g = torch.Generator().manual_seed(1)
        for it in range(5):
            xs = torch.randn(world * 8, 16, generator=g)
            ys = torch.randn(world * 8, 4, generator=g)
            opt.zero_grad()
            loss = torch.nn.functional.mse_loss(model(xs[rank * 8:(rank + 1) * 8]), ys[rank * 8:(rank + 1) * 8])
            loss.backward()
            opt.step()
            ropt.zero_grad()
            torch.nn.functional.mse_loss(ref(xs), ys).backward()
            ropt.step()
        for p, r in zip(net.parameters(), ref.parameters()):
            torch.testing.assert_close(p, r, rtol=1e-5, atol=1e-6)
        # Reducer: manual averaging
        t = torch.nn.Linear(4, 4)
        red = Reducer(t)
        t.weight.grad = torch.full_like(t.weight, float(rank))
        t.bias.grad = torch.full_like(t.bias, float(rank) * 2)
        red.reduce()
        assert torch.all(t.weight.grad == (world - 1) / 2.0)
        assert torch.all(t.bias.grad == (world - 1))
        # no_sync accumulates locally
        model.zero_grad()
        with model.no_sync():
            model(xs[:8]).sum().backward()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_ddp_matches_full_batch_training():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_equiv_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] == "ok" for r in res), res


def _zero_grad_worker(rank, world, port, q):
    try:
        _init(rank, world, port)
        from apex.optimizers import FusedSGD
        from apex.parallel import DistributedDataParallel as DDP

        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
        model = DDP(net, message_size=50)
        opt = FusedSGD(model.parameters(), lr=0.1)
        for i in range(3):
            opt.zero_grad()
            model(torch.randn(5, 8)).sum().backward()
            if i:
                # grads stay views of the one bucket buffer and are correct after a whole-buffer zero
                flat = net[0].weight._apex_bucket_flat
                assert all(p.grad.data_ptr() >= flat.data_ptr() for p in net.parameters())
            opt.step()
        opt.zero_grad()
        assert all(float(p.grad.abs().sum()) == 0.0 for p in net.parameters())
        assert net[0].weight._apex_bucket_flat._apex_nparams == 4
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_fused_optimizer_zero_grad_on_ddp_buckets():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_zero_grad_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] == "ok" for r in res), res


def _channels_last_worker(rank, world, port, q):
    try:
        _init(rank, world, port)
        from apex.parallel import DistributedDataParallel as DDP

        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.ReLU(), torch.nn.Conv2d(8, 4, 1))
        net = net.to(memory_format=torch.channels_last)
        model = DDP(net, message_size=100)
        for i in range(2):
            model.zero_grad(set_to_none=False)
            x = torch.randn(2, 3, 6, 6).to(memory_format=torch.channels_last) + rank
            model(x).sum().backward()
        w = net[0].weight
        # the grad is a bucket view that keeps the channels_last strides of its parameter
        assert w.grad.stride() == w.stride(), (w.grad.stride(), w.stride())
        ref = [torch.empty_like(w.grad) for _ in range(world)]
        dist.all_gather(ref, w.grad.contiguous())
        assert all(torch.equal(ref[0], r) for r in ref)
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_ddp_channels_last_params():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_channels_last_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] == "ok" for r in res), res
