"""Tensor-parallel backward overlap paths on CPU/gloo (TP=2), each against the serial layer pair:

* async input-gradient all-reduce in ColumnParallelLinear (the default) and the synchronous
  composition (``no_async_tensor_model_parallel_allreduce=True``) give the same gradients;
* ``gradient_accumulation_fusion`` accumulates dW into the fp32 ``main_grad`` across backward
  passes and leaves ``.grad`` unset;
* sequence parallelism: a column -> row pair on a sequence-sharded activation ([s/tp, b, h])
  matches the serial pair, output and input gradient still sharded;
* ``fusion_sync``: gradient_accumulation_fusion with the async all-reduce OFF — the column layer
  must still all-reduce dX (through copy_to_tensor_model_parallel_region);
* ``fusion_fp16``: ``accumulation_in_fp16`` accumulates into a 16-bit main_grad.
"""
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


def _pair(mode, seq_par=False):
    from apex.transformer import tensor_parallel as tp

    torch.manual_seed(0)
    fusion = mode.startswith("fusion")
    col = tp.ColumnParallelLinear(8, 16, gather_output=False, keep_master_weight_for_test=True,
                                  no_async_tensor_model_parallel_allreduce=(mode in ("sync", "fusion_sync")),
                                  gradient_accumulation_fusion=fusion, sequence_parallel_enabled=seq_par,
                                  accumulation_in_fp16=(mode == "fusion_fp16"))
    torch.manual_seed(1)
    row = tp.RowParallelLinear(16, 8, input_is_parallel=True, keep_master_weight_for_test=True,
                               gradient_accumulation_fusion=fusion, sequence_parallel_enabled=seq_par,
                               accumulation_in_fp16=(mode == "fusion_fp16"))
    with torch.no_grad():
        col.bias.uniform_(-1, 1)
        row.bias.uniform_(-1, 1)
    dist.broadcast(row.bias.data, 0)
    return col, row


def _full_col_bias(col, world):
    cb = [torch.empty_like(col.bias) for _ in range(world)]
    dist.all_gather(cb, col.bias.detach().contiguous())
    return torch.cat(cb)


def _overlap(rank, world, mode):
    from apex.transformer import parallel_state as ps

    ps.initialize_model_parallel(world, 1)
    col, row = _pair(mode)
    fusion = mode.startswith("fusion")
    mg_dtype = torch.float16 if mode == "fusion_fp16" else torch.float32
    if fusion:
        for m in (col, row):
            m.weight.main_grad = torch.zeros_like(m.weight, dtype=mg_dtype)
    cb = _full_col_bias(col, world)
    gw_ref = torch.zeros_like(col.master_weight)
    for it in range(2):
        torch.manual_seed(10 + it)
        x = torch.randn(5, 8, requires_grad=True)
        h, _ = col(x)
        y, _ = row(F.gelu(h))
        y.square().sum().backward()
        xr = x.detach().clone().requires_grad_(True)
        wc = col.master_weight.detach().clone().requires_grad_(True)
        yr = F.linear(F.gelu(F.linear(xr, wc, cb)), row.master_weight, row.bias.detach())
        yr.square().sum().backward()
        torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(x.grad, xr.grad, rtol=1e-5, atol=1e-5)
        gw_ref += wc.grad
    n = col.output_size_per_partition
    mine = gw_ref[rank * n:(rank + 1) * n]
    if fusion:
        assert col.weight.grad is None and row.weight.grad is None
        tol = 2e-2 if mode == "fusion_fp16" else 1e-5
        assert col.weight.main_grad.dtype == mg_dtype
        torch.testing.assert_close(col.weight.main_grad.float(), mine, rtol=tol, atol=tol)
    else:
        torch.testing.assert_close(col.weight.grad, mine, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("mode", ["async", "sync", "fusion", "fusion_sync", "fusion_fp16"])
def test_column_row_backward_overlap_modes(mode):
    _spawn(_overlap, 2, mode)


def _seqpar(rank, world):
    from apex.transformer import parallel_state as ps

    ps.initialize_model_parallel(world, 1)
    col, row = _pair("async", seq_par=True)
    cb = _full_col_bias(col, world)
    torch.manual_seed(3)
    S, B, H = 6, 3, 8
    x_full = torch.randn(S, B, H)
    x = x_full[rank * S // world:(rank + 1) * S // world].clone().requires_grad_(True)
    h, _ = col(x)
    y, bias = row(F.gelu(h))
    assert y.shape == (S // world, B, 8)
    (y.square().sum()).backward()
    xr = x_full.clone().requires_grad_(True)
    yr = F.linear(F.gelu(F.linear(xr, col.master_weight, cb)), row.master_weight, row.bias.detach())
    yr.square().sum().backward()
    sl = slice(rank * S // world, (rank + 1) * S // world)
    torch.testing.assert_close(y, yr[sl], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(x.grad, xr.grad[sl], rtol=1e-5, atol=1e-5)


def test_sequence_parallel_column_row_pair():
    _spawn(_seqpar, 2)
