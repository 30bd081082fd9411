"""Context parallelism on CPU/gloo (apex.transformer.context_parallel).

Every rank builds the same full-sequence q, k, v, takes its shard (zigzag or contiguous layout),
runs ring / Ulysses attention, and compares its output shard and its q/k/v gradient shards with
the single-process attention of the full sequence (fp32 torch composition): causal and not,
2 and 4 ranks. Also: the layouts round-trip through shard_sequence / gather_sequence, the CP
groups of parallel_state, and dropout runs with finite gradients.
"""
import os
import socket
import traceback

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


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


def _full_attention(q, k, v, causal, scale):
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) * scale
    if causal:
        S = s.shape[-1]
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool).triu(1), float("-inf"))
    return torch.einsum("bhqk,bkhd->bqhd", s.softmax(-1), v)


def _case(rank, world, kind, causal, layout):
    from apex.transformer import context_parallel as cp

    torch.manual_seed(0)
    B, S, H, D = 2, 8 * world, 4, 16
    q, k, v = (torch.randn(B, S, H, D, dtype=torch.float64) for _ in range(3))
    do = torch.randn(B, S, H, D, dtype=torch.float64)
    scale = 0.3
    qr, kr, vr = (t.clone().requires_grad_() for t in (q, k, v))
    ref = _full_attention(qr, kr, vr, causal, scale)
    ref.backward(do)
    g = dist.new_group(list(range(world)))
    shard = lambda t: cp.shard_sequence(t, g, layout)  # noqa: E731
    ql, kl, vl = (shard(t).clone().requires_grad_() for t in (q, k, v))
    if kind == "ring":
        out = cp.ring_attention(ql, kl, vl, group=g, causal=causal, scale=scale, layout=layout)
    else:
        out = cp.ulysses_attention(ql, kl, vl, group=g, causal=causal, scale=scale)
    out.backward(shard(do))
    # ring: fp64 end to end; Ulysses' local attention is apex's reference composition (fp32 softmax)
    tol = dict(atol=1e-9, rtol=1e-7) if kind == "ring" else dict(atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(out, shard(ref.detach()), **tol)
    for got, want in ((ql.grad, qr.grad), (kl.grad, kr.grad), (vl.grad, vr.grad)):
        torch.testing.assert_close(got, shard(want), **tol)
    # the shards reassemble into the full sequence
    torch.testing.assert_close(cp.gather_sequence(out.detach(), g, layout), ref.detach(), **tol)


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("layout", ["zigzag", "contiguous"])
def test_ring_attention_matches_full(world, causal, layout):
    _spawn(_case, world, "ring", causal, layout)


@pytest.mark.parametrize("causal", [False, True])
def test_ulysses_attention_matches_full(causal):
    _spawn(_case, 2, "ulysses", causal, "contiguous")


def _groups_and_dropout(rank, world):
    from apex.transformer import context_parallel as cp
    from apex.transformer import parallel_state as ps

    # world 4: TP 1, PP 1, DP 4 -> CP groups of 2 consecutive DP ranks
    ps.initialize_model_parallel(1, 1, context_parallel_size_=2)
    assert ps.get_context_parallel_world_size() == 2
    assert ps.get_context_parallel_global_ranks() == [rank // 2 * 2, rank // 2 * 2 + 1]
    assert ps.get_context_parallel_rank() == rank % 2
    assert ps.get_data_parallel_world_size() == 4
    torch.manual_seed(rank // 2)  # one sample per CP group
    q, k, v = (torch.randn(1, 8, 2, 8, requires_grad=True) for _ in range(3))
    out = cp.ring_attention(q, k, v, causal=True, dropout_p=0.2)  # the default (parallel_state) group
    out.float().sum().backward()
    assert torch.isfinite(out).all() and all(torch.isfinite(t.grad).all() for t in (q, k, v))


def test_context_parallel_groups_and_dropout():
    _spawn(_groups_and_dropout, 4)


@pytest.mark.parametrize("causal", [False, True])
def test_ring_attention_cp1_without_process_group(causal):
    """CP size 1 with torch.distributed NOT initialised and no parallel_state: ring_attention falls
    back to a one-rank ring (no send to itself in the backward) and matches full attention."""
    from apex.transformer import context_parallel as cp

    assert not dist.is_initialized()
    torch.manual_seed(3)
    q, k, v = (torch.randn(2, 16, 2, 8, dtype=torch.float64) for _ in range(3))
    leaves = [t.clone().requires_grad_() for t in (q, k, v)]
    ref = [t.clone().requires_grad_() for t in (q, k, v)]
    out = cp.ring_attention(*leaves, causal=causal)
    want = _full_attention(*ref, causal, 1.0 / 8 ** 0.5)
    torch.testing.assert_close(out, want)
    do = torch.randn_like(out)
    out.backward(do)
    want.backward(do)
    for a, b in zip(leaves, ref):
        torch.testing.assert_close(a.grad, b.grad)


def test_merge_into_row_range_matches_whole_merge():
    """_merge with a row offset (a zigzag step that reaches only the late chunk merges into that half
    of the accumulator) equals merging the same block padded to all rows with -inf elsewhere."""
    from apex.transformer import context_parallel as cp

    g = torch.Generator().manual_seed(0)
    B, S, H, D = 2, 8, 3, 16
    o0 = torch.randn(B, S, H, D, generator=g, dtype=torch.float64)
    l0 = torch.randn(B, H, S, generator=g, dtype=torch.float64)
    o1 = torch.randn(B, S // 2, H, D, generator=g, dtype=torch.float64)
    l1 = torch.randn(B, H, S // 2, generator=g, dtype=torch.float64)
    l1[0, 1, 2] = float("inf")  # a row with no visible key in this block (flash marks it +inf)
    acc_o, acc_l = cp._merge(None, None, o0, l0, 0, S)
    acc_o, acc_l = cp._merge(acc_o, acc_l, o1, l1, S // 2, S)
    # reference: the block padded to all rows, -inf (no contribution) on the early half
    op = torch.cat([torch.zeros_like(o1), o1], dim=1)
    lp = torch.cat([torch.full_like(l1, float("-inf")), torch.where(torch.isposinf(l1), torch.full_like(l1, float("-inf")), l1)], dim=2)
    ref_l = torch.logaddexp(l0, lp)
    w0 = torch.exp(l0 - ref_l).transpose(1, 2).unsqueeze(-1)
    w1 = torch.exp(lp - ref_l).transpose(1, 2).unsqueeze(-1)
    ref_o = o0 * w0 + op * w1
    torch.testing.assert_close(acc_l, ref_l)
    torch.testing.assert_close(acc_o, ref_o)
    # first block covering only part of the rows: the rest stay empty (lse -inf, output 0)
    a_o, a_l = cp._merge(None, None, o1, l1, S // 2, S)
    assert torch.isneginf(a_l[:, :, : S // 2]).all() and float(a_o[:, : S // 2].abs().max()) == 0.0
