"""DDP fp32_main_grad mode on CPU/gloo (world 2): a bf16 model accumulates 8 micro-batches under
no_sync(); every parameter's gradient lives in an fp32 ``main_grad`` (views of fp32 buckets),
``.grad`` stays None, the last micro-batch's backward all-reduces the fp32 buckets, and the
result equals the fp32 sum of the per-micro-batch gradients averaged over ranks (where plain
bf16 ``.grad`` accumulation would have rounded after every add). The fused optimizer then
consumes main_grad and zero_grad zero-fills it. GPU path (fused fp32-accumulating weight-gradient
GEMMs): tests/test_main_grad_gpu.py."""
import os
import socket
import traceback

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.set_num_threads(1)
        from apex.optimizers import FusedAdam
        from apex.parallel import DistributedDataParallel as DDP

        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 8)).to(torch.bfloat16)
        ref_params = [p.detach().clone() for p in net.parameters()]
        model = DDP(net, message_size=200, fp32_main_grad=True)
        for p in net.parameters():
            assert p.main_grad.dtype == torch.float32 and p.grad is None
        g = torch.Generator().manual_seed(5)
        xs = [torch.randn(world * 4, 16, generator=g).to(torch.bfloat16) for _ in range(8)]
        # reference: fp32 sum of each micro-batch's bf16 gradient, averaged over ranks
        ref = [torch.zeros(p.shape, dtype=torch.float32) for p in net.parameters()]
        twin = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 8)).to(torch.bfloat16)
        with torch.no_grad():
            for tp, rp in zip(twin.parameters(), ref_params):
                tp.copy_(rp)
        for mb, x in enumerate(xs):
            for r in range(world):
                twin.zero_grad()
                twin(x[r * 4:(r + 1) * 4]).float().pow(2).sum().backward()
                for a, tp in zip(ref, twin.parameters()):
                    a.add_(tp.grad.float() / world)
        for mb, x in enumerate(xs):
            last = mb == len(xs) - 1
            ctx = model.no_sync() if not last else torch.autograd.graph.saved_tensors_hooks(lambda t: t, lambda t: t)
            with ctx:
                model(x[rank * 4:(rank + 1) * 4]).float().pow(2).sum().backward()
            for p in net.parameters():
                assert p.grad is None
        for p, a in zip(net.parameters(), ref):
            torch.testing.assert_close(p.main_grad, a, rtol=1e-5, atol=1e-5)
        # bf16 accumulation of the same micro-batch gradients differs (rounding at every add)
        acc16 = [torch.zeros(p.shape, dtype=torch.bfloat16) for p in net.parameters()]
        for x in xs:
            for r in range(world):
                twin.zero_grad()
                twin(x[r * 4:(r + 1) * 4]).float().pow(2).sum().backward()
                for a, tp in zip(acc16, twin.parameters()):
                    a.add_(tp.grad / world)
        worst16 = max(float((a.float() - r_).abs().max()) for a, r_ in zip(acc16, ref))
        worst32 = max(float((p.main_grad - r_).abs().max()) for p, r_ in zip(net.parameters(), ref))
        assert worst32 < worst16, (worst32, worst16)
        opt = FusedAdam(net.parameters(), lr=1e-3)
        before = [p.detach().clone() for p in net.parameters()]
        opt.step()
        assert any(not torch.equal(b, p.detach()) for b, p in zip(before, net.parameters()))
        opt.zero_grad()
        assert all(float(p.main_grad.abs().max()) == 0.0 for p in net.parameters())
        q.put((rank, "ok"))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_fp32_main_grad_accumulation():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    assert all(r[1] == "ok" for r in res), res


class _FusedAccum(torch.autograd.Function):
    """Stands in for a fused weight-gradient producer on the CPU: accumulates dW into
    weight.main_grad and hands autograd the ZeroTensor placeholder (apex.ops.fused)."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x @ w.t()

    @staticmethod
    def backward(ctx, dy):
        from apex.ops.fused import main_grad_placeholder

        x, w = ctx.saved_tensors
        w.main_grad.add_(dy.t().float() @ x.float())
        return dy @ w, main_grad_placeholder(w)


def _tied_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.set_num_threads(1)
        from apex.parallel import DistributedDataParallel as DDP

        class Tied(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.emb = torch.nn.Embedding(12, 8)

            def forward(self, ids):
                h = self.emb(ids)  # lookup: an ordinary dense gradient for the shared weight
                return _FusedAccum.apply(h, self.emb.weight)  # tied head: fused main_grad producer

        torch.manual_seed(0)
        net = Tied()
        twin = Tied()
        twin.load_state_dict(net.state_dict())
        model = DDP(net, message_size=50, fp32_main_grad=True)
        g = torch.Generator().manual_seed(1)
        ids = [torch.randint(0, 12, (world * 3,), generator=g) for _ in range(3)]
        for mb, x in enumerate(ids):
            with (model.no_sync() if mb < len(ids) - 1 else torch.enable_grad()):
                model(x[rank * 3:(rank + 1) * 3]).pow(2).sum().backward()
        ref = torch.zeros(12, 8)
        for x in ids:
            for r in range(world):
                twin.zero_grad()
                out = twin.emb(x[r * 3:(r + 1) * 3]) @ twin.emb.weight.t()
                out.pow(2).sum().backward()
                ref += twin.emb.weight.grad / world
        torch.testing.assert_close(net.emb.weight.main_grad, ref, rtol=1e-5, atol=1e-5)
        assert net.emb.weight.grad is None
        q.put((rank, "ok"))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_fp32_main_grad_tied_weight_keeps_other_uses():
    """A weight with a fused main_grad producer AND another use (tied embedding / LM head): the
    other use's gradient is summed with the placeholder by autograd and must reach main_grad."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_tied_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    assert all(r[1] == "ok" for r in res), res


class _Crossed(torch.nn.Module):
    """Registered a, b, c but used as a(c(b(x))): grads become ready a, c, b — not the reverse
    registration order c, b, a the provisional main_grad layout assumes."""

    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(8, 8, bias=False)
        self.b = torch.nn.Linear(8, 8, bias=False)
        self.c = torch.nn.Linear(8, 8, bias=False)

    def forward(self, x):
        return self.a(torch.tanh(self.c(torch.tanh(self.b(x)))))


def _order_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.set_num_threads(1)
        from apex.parallel import DistributedDataParallel as DDP

        torch.manual_seed(0)
        net = _Crossed()
        arrived = []
        for name, p in net.named_parameters():  # registered before DDP's hooks: runs first
            p.register_post_accumulate_grad_hook(lambda p, n=name.split(".")[0]: arrived.append(n))
        model = DDP(net, message_size=64, fp32_main_grad=True)  # one 8x8 weight per bucket
        names = {id(p): n.split(".")[0] for n, p in net.named_parameters()}
        launches = []
        orig = model._start_bucket

        def spy(b, lane):
            launches.append(([names[id(model._params[i])] for i in b.params], len(arrived)))
            return orig(b, lane)

        model._start_bucket = spy
        x = torch.randn(4, 8)
        for it in range(3):
            arrived.clear()
            launches.clear()
            model.zero_grad()
            model(x + rank).pow(2).sum().backward()
            assert arrived == ["a", "c", "b"], arrived
            mg = {n: p.main_grad.clone() for n, p in net.named_parameters()}
            if it == 0:
                # first backward: order recorded, buffers re-laid out in it, values carried over
                layout = [[names[id(model._params[i])] for i in bk.params] for bk in model._buckets]
                assert layout == [["a"], ["c"], ["b"]], layout
            else:
                # steady state: bucket k goes on the wire as soon as the k-th gradient is ready
                assert launches == [(["a"], 1), (["c"], 2), (["b"], 3)], launches
            # against plain fp32 autograd averaged over ranks
            twin = _Crossed()
            twin.load_state_dict(net.state_dict())
            tot = {n: torch.zeros_like(p) for n, p in twin.named_parameters()}
            for r in range(world):
                twin.zero_grad()
                twin(x + r).pow(2).sum().backward()
                for n, p in twin.named_parameters():
                    tot[n] += p.grad / world
            for n in tot:
                torch.testing.assert_close(mg[n], tot[n], rtol=1e-5, atol=1e-6)
        # torch.optim reads p.grad (None in main_grad mode): the guard raises instead of a silent no-op
        opt = torch.optim.SGD(net.parameters(), lr=0.1)
        try:
            opt.step()
            raise AssertionError("torch.optim step on main_grad params did not raise")
        except RuntimeError as e:
            assert "main_grad" in str(e)
        q.put((rank, "ok"))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_fp32_main_grad_layout_follows_grad_ready_order():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_order_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    assert all(r[1] == "ok" for r in res), res
