"""apex DDP options and layout, CPU only (gloo world 2-3, fake process group world 8).

* rank-0 bucket structure broadcast (reference apex/parallel/distributed.py:176-203): ranks whose
  autograd produces gradients in DIFFERENT orders must still agree on one bucket layout, or
  the in-order bucket all-reduces would average unrelated parameters;
* allreduce_always_fp32, gradient_predivide_factor, num_allreduce_streams (several
  communicators), allreduce_trigger_params, comm_stats();
* fake_pg world 8: the bucket cut points for message_size / first_bucket_size.
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


def _run(world, target, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] == "ok" for r in res), res


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)


class _Branches(torch.nn.Module):
    """out = sum_i c_i * (x * p_i).sum(), branches evaluated in a rank-dependent order so the
    AccumulateGrad hooks fire in a different order on every rank."""

    def __init__(self, n, k, order):
        super().__init__()
        self.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.ones(n)) for _ in range(k)])
        self.order = order

    def forward(self, x):
        out = 0
        for i in self.order:
            out = out + float(i + 1) * (x * self.ps[i]).sum()
        return out


def _order_worker(rank, world, port, q):
    try:
        _init(rank, world, port)
        from apex.parallel import DistributedDataParallel as DDP

        k, n = 5, 64
        order = list(range(k)) if rank % 2 == 0 else list(reversed(range(k)))
        model = DDP(_Branches(n, k, order), message_size=1)
        for it in range(4):
            model.zero_grad(set_to_none=False)
            x = torch.full((n,), float(it + rank))
            model(x).backward()
            mean_x = it + (world - 1) / 2.0
            for i, p in enumerate(model.module.ps):
                assert torch.all(p.grad == (i + 1) * mean_x), (rank, it, i, p.grad[:2])
        # every rank holds rank 0's layout (param order of the buckets)
        lay = torch.tensor([b.params[0] for b in model._buckets])
        ref = lay.clone()
        dist.broadcast(ref, 0)
        assert torch.equal(lay, ref), (lay, ref)
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_rank0_bucket_structure_wins(world):
    _run(world, _order_worker)


def _options_worker(rank, world, port, q, opts):
    try:
        _init(rank, world, port)
        from apex.parallel import DistributedDataParallel as DDP

        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Tanh(), torch.nn.Linear(16, 4))
        ref = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Tanh(), torch.nn.Linear(16, 4))
        ref.load_state_dict(net.state_dict())
        kw = dict(opts)
        if kw.pop("trigger", False):
            kw["allreduce_trigger_params"] = [net[0].weight]  # the last grad to arrive
        model = DDP(net, message_size=40, **kw)
        g = torch.Generator().manual_seed(3)
        for it in range(3):
            xs = torch.randn(world * 4, 8, generator=g)
            model.zero_grad()
            model(xs[rank * 4:(rank + 1) * 4]).pow(2).sum().backward()
            ref.zero_grad()
            (ref(xs).pow(2).sum() / world).backward()
            for p, r in zip(net.parameters(), ref.parameters()):
                torch.testing.assert_close(p.grad, r.grad, rtol=1e-5, atol=1e-6)
        st = model.comm_stats()
        assert st["num_buckets"] == len(model._buckets) and st["backend"] == "gloo"
        assert sum(st["bucket_bytes"]) == sum(p.numel() * 4 for p in net.parameters())
        if "num_allreduce_streams" in opts:
            assert st["num_communicators"] == opts["num_allreduce_streams"]
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("opts", [
    {"allreduce_always_fp32": True},
    {"gradient_predivide_factor": 2.0},
    {"num_allreduce_streams": 3},
    {"trigger": True},
    {"delay_allreduce": True, "allreduce_always_fp32": True},
])
def test_ddp_options_match_full_batch(opts):
    _run(2, _options_worker, opts)


def test_fp32_allreduce_of_bf16_grads():
    _run(2, _bf16_worker)


def _bf16_worker(rank, world, port, q):
    try:
        _init(rank, world, port)
        from apex.parallel import DistributedDataParallel as DDP

        p = torch.nn.Parameter(torch.ones(256, dtype=torch.bfloat16))

        class M(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.p = p

            def forward(self, x):
                return (x * self.p).sum()

        model = DDP(M(), allreduce_always_fp32=True, message_size=1)
        for it in range(2):
            model.zero_grad(set_to_none=False)
            # values whose bf16 SUM would round but whose fp32 average is exact in bf16
            x = torch.full((256,), 1.0 + rank * 2.0 ** -7, dtype=torch.bfloat16)
            model(x).backward()
            assert p.grad.dtype == torch.bfloat16
            want = 1.0 + (world - 1) / 2.0 * 2.0 ** -7
            assert torch.all(p.grad.float() == torch.tensor(want, dtype=torch.bfloat16).float()), p.grad[:3]
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


# ----------------------------------------------------------------------------- fake pg, world 8
@pytest.fixture
def fake_world8():
    from torch.testing._internal.distributed.fake_pg import FakeStore

    dist.init_process_group("fake", store=FakeStore(), rank=5, world_size=8)
    yield
    dist.destroy_process_group()


def test_bucket_layout_world8(fake_world8):
    from apex.parallel import DistributedDataParallel as DDP

    sizes = [100, 300, 50, 700, 20, 400]
    params = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(n)) for n in sizes])

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.params = params

        def forward(self):
            return sum((p * (i + 1)).sum() for i, p in enumerate(self.params))

    model = DDP(M(), message_size=500, first_bucket_size=150)
    assert model.world_size == 8
    model().backward()
    # grad-ready order is reverse of use: params 5,4,3,2,1,0 (sizes 400,20,700,50,300,100)
    got = [(b.numel, [sizes[i] for i in b.params]) for b in model._buckets]
    # first bucket cut at >=150 elements, then every >=500; every slot starts on a 16-byte
    # boundary (fp32: 4 elements), so the 50-element grad is followed by 2 padding elements
    assert got == [(400, [400]), (720, [20, 700]), (452, [50, 300, 100])], got
    # grads are views of one flat buffer laid out in bucket order
    flat = model.allreduce_buffers[0]
    assert flat.numel() == sum(sizes) + 2
    assert all(p.grad.data_ptr() % 16 == 0 for p in params)
    for i, p in enumerate(params):
        assert p.grad.data_ptr() >= flat.data_ptr()
        # the fake collective sums nothing, so the average leaves grad / world
        torch.testing.assert_close(p.grad, torch.full_like(p, (i + 1) / 8.0))
    # second iteration: steady-state path, every bucket fires exactly once
    model.zero_grad(set_to_none=False)
    model().backward()
    assert model._next_bucket == len(model._buckets)
    st = model.comm_stats()
    assert st["world_size"] == 8 and st["num_buckets"] == 3
    assert st["bucket_bytes"] == [400 * 4, 720 * 4, 452 * 4]


def test_broadcast_layout_from_rank0_world8(fake_world8, monkeypatch):
    """Rank 5 records its own grad-ready order but adopts rank 0's (the structure broadcast)."""
    from apex.parallel import DistributedDataParallel as DDP

    params = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(10)) for _ in range(4)])

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.params = params

        def forward(self):
            return sum(p.sum() for p in self.params)

    rank0_order = [2, 0, 3, 1]
    real_bcast = dist.broadcast

    def fake_bcast(t, src, group=None, **kw):
        if t.dtype == torch.int64 and t.numel() == 4:
            t.copy_(torch.tensor(rank0_order))
        return real_bcast(t, src, group=group, **kw)

    monkeypatch.setattr(dist, "broadcast", fake_bcast)
    model = DDP(M(), message_size=1)
    model().backward()
    assert [b.params for b in model._buckets] == [[i] for i in rank0_order]


def test_allreduce_sweep_tool_gloo():
    """tools/allreduce_sweep.py end to end under torchrun (gloo, 2 ranks, tiny sizes)."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, APEX_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(root, "tools", "allreduce_sweep.py"), "--cpu", "--min-mb", "0.25",
                        "--max-mb", "0.5", "--comms", "1,2", "--iters", "2", "--dtypes", "fp32"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    rows = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(rows) == 4 and all(x["busbw_gbs"] > 0 and x["world"] == 2 for x in rows), rows


def _subgroup_lanes_worker(rank, world, port, q):
    """Two disjoint DP groups {0,1} and {2,3}, each DDP with 2 communicator lanes: every rank
    must create every group's lanes (dist.new_group is collective over the default group), and
    each group's gradients average only over its own two ranks."""
    try:
        _init(rank, world, port)
        from apex.parallel import DistributedDataParallel as DDP

        groups = [dist.new_group([0, 1]), dist.new_group([2, 3])]
        mine = groups[rank // 2]
        torch.manual_seed(rank // 2)  # the two DP groups hold different models
        net = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Tanh(), torch.nn.Linear(16, 4))
        ref = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Tanh(), torch.nn.Linear(16, 4))
        ref.load_state_dict(net.state_dict())
        model = DDP(net, message_size=40, process_group=mine, num_allreduce_streams=2)
        assert model.comm_stats()["num_communicators"] == 2
        g = torch.Generator().manual_seed(7 + rank // 2)
        for _ in range(2):
            xs = torch.randn(8, 8, generator=g)
            model.zero_grad()
            model(xs[(rank % 2) * 4:(rank % 2 + 1) * 4]).pow(2).sum().backward()
            ref.zero_grad()
            (ref(xs).pow(2).sum() / 2).backward()
            for p, r in zip(net.parameters(), ref.parameters()):
                torch.testing.assert_close(p.grad, r.grad, rtol=1e-5, atol=1e-6)
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_ddp_lanes_on_dp_subgroups():
    _run(4, _subgroup_lanes_worker)
