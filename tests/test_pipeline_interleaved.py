"""Interleaved 1F1B pipeline schedule (virtual pipeline stages) on CPU/gloo, against the same
network run serially in one process: losses and every gradient must match, and the schedule
must really interleave — its peak number of stored forward units stays well under the n*V of an
all-forwards-then-all-backwards (GPipe) order."""
import os
import socket
import traceback

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(fn, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_wrap, args=(fn, r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] == "ok" for r in res), res


def _wrap(fn, rank, world, port, q, *args):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.set_num_threads(1)
        fn(rank, world, *args)
        q.put((rank, "ok"))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        from apex.transformer import parallel_state as ps

        ps.destroy_model_parallel()
        dist.destroy_process_group()


class _Chunk(torch.nn.Module):
    def __init__(self, w, b):
        super().__init__()
        self.lin = torch.nn.Linear(6, 6)
        with torch.no_grad():
            self.lin.weight.copy_(w)
            self.lin.bias.copy_(b)
        self.input_tensor = None

    def set_input_tensor(self, t):
        self.input_tensor = t

    def forward(self, x):
        inp = x if self.input_tensor is None else self.input_tensor
        return torch.tanh(self.lin(inp))


def _interleaved(rank, world, V, n_micro):
    from apex.transformer import parallel_state as ps
    from apex.transformer.pipeline_parallel import get_forward_backward_func, setup_microbatch_calculator
    from apex.transformer.pipeline_parallel.schedules import last_schedule_stats

    P = world
    ps.initialize_model_parallel(1, P, virtual_pipeline_model_parallel_size_=V)
    mb = 2
    setup_microbatch_calculator(rank, None, n_micro * mb, mb, 1)
    torch.manual_seed(0)
    weights = [(torch.randn(6, 6) * 0.6, torch.randn(6) * 0.1) for _ in range(P * V)]
    data = torch.randn(n_micro * mb, 6)
    target = torch.randn(n_micro * mb, 6)
    # rank r holds virtual stages c*P + r for c = 0..V-1
    chunks = [_Chunk(*weights[c * P + rank]) for c in range(V)]
    tgt = list(target.chunk(n_micro))
    seen = {"i": 0}

    def fwd_step(batch, m):
        out = m(batch)

        def loss_fn(o):
            t = tgt[seen["i"] % n_micro]
            seen["i"] += 1
            loss = F.mse_loss(o, t)
            return loss, {"loss": loss.detach()}

        return out, loss_fn

    fb = get_forward_backward_func(V, P)
    losses = fb(fwd_step, data, chunks, forward_only=False, tensor_shape=(mb, 6), dtype=torch.float32)
    st = last_schedule_stats()
    # serial reference over all P*V stages
    ref = [_Chunk(*w) for w in weights]
    total = 0.0
    for xb, tb in zip(data.chunk(n_micro), target.chunk(n_micro)):
        h = xb
        for s in ref:
            h = s(h)
        loss = F.mse_loss(h, tb) / n_micro
        loss.backward()
        total += float(loss)
    for c in range(V):
        r = ref[c * P + rank]
        torch.testing.assert_close(chunks[c].lin.weight.grad, r.lin.weight.grad, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(chunks[c].lin.bias.grad, r.lin.bias.grad, rtol=1e-5, atol=1e-6)
    if rank == P - 1:
        assert len(losses) == n_micro
        assert abs(sum(float(l["loss"]) for l in losses) / n_micro - total) < 1e-5
    assert st["units"] == n_micro * V
    if n_micro > P:  # 1F1B part exists: fewer live units than GPipe's n*V
        assert st["max_live"] <= st["warmup"] + 1 < n_micro * V, st


@pytest.mark.parametrize("world,V,n_micro", [(2, 2, 4), (2, 2, 8), (4, 2, 8), (2, 3, 2), (3, 2, 6)])
def test_interleaved_1f1b_matches_serial(world, V, n_micro):
    _spawn(_interleaved, world, V, n_micro)


def _bad_micro(rank, world):
    from apex.transformer import parallel_state as ps
    from apex.transformer.pipeline_parallel import get_forward_backward_func, setup_microbatch_calculator

    ps.initialize_model_parallel(1, world, virtual_pipeline_model_parallel_size_=2)
    setup_microbatch_calculator(rank, None, 3 * 2, 2, 1)
    fb = get_forward_backward_func(2, world)
    with pytest.raises(RuntimeError, match="multiple of"):
        fb(lambda b, m: (m(b), None), torch.randn(6, 6), [_Chunk(torch.eye(6), torch.zeros(6))] * 2,
           tensor_shape=(2, 6))


def test_interleaved_rejects_bad_microbatch_count():
    _spawn(_bad_micro, 2)


def _pp_dp(rank, world, V):
    """PP=2 x DP=2 (world 4): every chunk wrapped in apex DDP over its data-parallel group. The
    schedules keep the hooks off until each chunk's last microbatch backward, so the bucket
    all-reduce runs once per step and the grads equal the serial full-batch average."""
    from apex.parallel import DistributedDataParallel as DDP
    from apex.transformer import parallel_state as ps
    from apex.transformer.pipeline_parallel import get_forward_backward_func, setup_microbatch_calculator

    P, DP = 2, 2
    ps.initialize_model_parallel(1, P, virtual_pipeline_model_parallel_size_=V if V > 1 else None)
    n_micro, mb = 4, 2
    setup_microbatch_calculator(rank, None, n_micro * mb * DP, mb, DP)
    torch.manual_seed(0)
    weights = [(torch.randn(6, 6) * 0.6, torch.randn(6) * 0.1) for _ in range(P * V)]
    data = torch.randn(DP, n_micro * mb, 6)
    target = torch.randn(DP, n_micro * mb, 6)
    pr, dr = ps.get_pipeline_model_parallel_rank(), ps.get_data_parallel_rank()
    chunks = [DDP(_Chunk(*weights[c * P + pr]), message_size=10, process_group=ps.get_data_parallel_group())
              for c in range(V)]
    tgt = list(target[dr].chunk(n_micro))
    seen = {"i": 0}

    def fwd_step(batch, m):
        out = m(batch)

        def loss_fn(o):
            t = tgt[seen["i"] % n_micro]
            seen["i"] += 1
            loss = F.mse_loss(o, t)
            return loss, {"loss": loss.detach()}

        return out, loss_fn

    fb = get_forward_backward_func(V if V > 1 else None, P)
    for _ in range(2):  # second step: steady-state buckets
        for ch in chunks:
            ch.zero_grad()
        seen["i"] = 0
        fb(fwd_step, data[dr], chunks if V > 1 else chunks[0], forward_only=False, tensor_shape=(mb, 6),
           dtype=torch.float32)
    ref = [_Chunk(*w) for w in weights]
    for d in range(DP):
        for xb, tb in zip(data[d].chunk(n_micro), target[d].chunk(n_micro)):
            h = xb
            for s in ref:
                h = s(h)
            (F.mse_loss(h, tb) / n_micro / DP).backward()
    for c in range(V):
        r = ref[c * P + pr]
        torch.testing.assert_close(chunks[c].module.lin.weight.grad, r.lin.weight.grad, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(chunks[c].module.lin.bias.grad, r.lin.bias.grad, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("V", [1, 2])
def test_pipeline_with_ddp_over_data_parallel_group(V):
    _spawn(_pp_dp, 4, V)
