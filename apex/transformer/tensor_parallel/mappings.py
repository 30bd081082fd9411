"""Autograd-aware TP communication primitives (NS-08).

  copy_to_tensor_model_parallel_region      fwd identity   / bwd all-reduce
  reduce_from_tensor_model_parallel_region  fwd all-reduce / bwd identity
  scatter_to_tensor_model_parallel_region   fwd split last dim / bwd all-gather
  gather_from_tensor_model_parallel_region  fwd all-gather last dim / bwd split
  scatter_to_sequence_parallel_region       fwd split first dim / bwd all-gather
  gather_from_sequence_parallel_region      fwd all-gather first dim / bwd reduce-scatter
  reduce_scatter_to_sequence_parallel_region fwd reduce-scatter first dim / bwd all-gather
All over RCCL (torch.distributed) within the TP group; first-dim collectives use the
single-buffer ``all_gather_into_tensor`` / ``reduce_scatter_tensor`` forms.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import parallel_state as ps
from .utils import split_tensor_along_last_dim


def _reduce(x):
    if ps.get_tensor_model_parallel_world_size() == 1:
        return x
    dist.all_reduce(x, group=ps.get_tensor_model_parallel_group())
    return x


def _split_last(x):
    ws = ps.get_tensor_model_parallel_world_size()
    if ws == 1:
        return x
    return split_tensor_along_last_dim(x, ws)[ps.get_tensor_model_parallel_rank()].contiguous()


def _gather_last(x):
    ws = ps.get_tensor_model_parallel_world_size()
    if ws == 1:
        return x
    x = x.contiguous()
    out = torch.empty((ws,) + tuple(x.shape), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out.view(ws * x.shape[0], *x.shape[1:]) if x.dim() else out, x,
                                group=ps.get_tensor_model_parallel_group())
    return torch.cat(out.unbind(0), dim=-1).contiguous()


def _split_first(x):
    ws = ps.get_tensor_model_parallel_world_size()
    if ws == 1:
        return x
    n = x.shape[0] // ws
    r = ps.get_tensor_model_parallel_rank()
    return x[r * n:(r + 1) * n].contiguous()


def _gather_first(x):
    ws = ps.get_tensor_model_parallel_world_size()
    if ws == 1:
        return x
    x = x.contiguous()
    out = torch.empty((ws * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x, group=ps.get_tensor_model_parallel_group())
    return out


def _reduce_scatter_first(x):
    ws = ps.get_tensor_model_parallel_world_size()
    if ws == 1:
        return x
    x = x.contiguous()
    out = torch.empty((x.shape[0] // ws,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.reduce_scatter_tensor(out, x, group=ps.get_tensor_model_parallel_group())
    return out


class _CopyToModelParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x

    @staticmethod
    def backward(ctx, g):
        # the all-reduce runs in place, so it works on a copy of the incoming gradient; at TP = 1
        # there is no collective and no copy (5 [tokens, hidden] clones per layer otherwise)
        return g if ps.get_tensor_model_parallel_world_size() == 1 else _reduce(g.clone())


class _ReduceFromModelParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x if ps.get_tensor_model_parallel_world_size() == 1 else _reduce(x.clone())

    @staticmethod
    def backward(ctx, g):
        return g


class _ScatterToModelParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return _split_last(x)

    @staticmethod
    def backward(ctx, g):
        return _gather_last(g)


class _GatherFromModelParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return _gather_last(x)

    @staticmethod
    def backward(ctx, g):
        return _split_last(g)


class _ScatterToSequenceParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return _split_first(x)

    @staticmethod
    def backward(ctx, g):
        return _gather_first(g)


class _GatherFromSequenceParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, to_model_parallel=True):
        ctx.to_model_parallel = to_model_parallel
        return _gather_first(x)

    @staticmethod
    def backward(ctx, g):
        if ctx.to_model_parallel:
            return _reduce_scatter_first(g), None
        return _split_first(g), None


class _ReduceScatterToSequenceParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return _reduce_scatter_first(x)

    @staticmethod
    def backward(ctx, g):
        return _gather_first(g)


def copy_to_tensor_model_parallel_region(x):
    return _CopyToModelParallelRegion.apply(x)


def reduce_from_tensor_model_parallel_region(x):
    return _ReduceFromModelParallelRegion.apply(x)


def scatter_to_tensor_model_parallel_region(x):
    return _ScatterToModelParallelRegion.apply(x)


def gather_from_tensor_model_parallel_region(x):
    return _GatherFromModelParallelRegion.apply(x)


def scatter_to_sequence_parallel_region(x):
    return _ScatterToSequenceParallelRegion.apply(x)


def gather_from_sequence_parallel_region(x, to_model_parallel=True):
    return _GatherFromSequenceParallelRegion.apply(x, to_model_parallel)


def reduce_scatter_to_sequence_parallel_region(x):
    return _ReduceScatterToSequenceParallelRegion.apply(x)
