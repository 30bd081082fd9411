"""Tensor-parallel layers (NS-08): ColumnParallelLinear, RowParallelLinear,
VocabParallelEmbedding.

Column-parallel splits the output features across the TP group (W row blocks), so the
forward needs no communication and the backward one all-reduce of the input gradient;
row-parallel splits the input features (W column blocks) and all-reduces the partial
outputs in the forward. A column -> row pair (attention QKV -> out-proj, MLP fc1 -> fc2)
therefore costs exactly one all-reduce forward and one backward per block — on MI355X
that is one RCCL ring over the TP group's direct xGMI links per sublayer.
With ``sequence_parallel_enabled`` the all-reduces become reduce-scatter / all-gather
along the sequence dimension (activations stay sharded between blocks).
GEMMs + bias use apex.ops.fused.fused_dense (bias grad via HIP colsum).

Backward overlap (``LinearWithGradAccumulationAndAsyncCommunication``, Megatron semantics):
  * async TP all-reduce (column-parallel, default on; ``no_async_tensor_model_parallel_allreduce``
    turns it off): the input gradient dX = dY W is computed first and its all-reduce (or, under
    sequence parallelism, its reduce-scatter) is launched asynchronously; the weight-gradient
    GEMM dW = dY^T X runs while RCCL moves dX over xGMI, and the wait comes last;
  * ``gradient_accumulation_fusion``: dW is accumulated straight into the parameter's fp32
    ``main_grad`` buffer (hipBLASLt with fp32 output, no bf16 dW tensor, no separate add); the
    weight then gets no ``.grad`` from autograd;
  * sequence parallel: the all-gather of the sequence-sharded input is redone in backward
    instead of keeping the gathered activation alive.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F
from torch import nn
from torch.nn.parameter import Parameter

import torch.distributed as dist

from ...ops import fused as fops
from .. import parallel_state as ps
from .mappings import (copy_to_tensor_model_parallel_region, gather_from_sequence_parallel_region,
                       gather_from_tensor_model_parallel_region, reduce_from_tensor_model_parallel_region,
                       reduce_scatter_to_sequence_parallel_region, scatter_to_tensor_model_parallel_region)
from .random import get_cuda_rng_tracker
from .utils import VocabUtility, divide

_MODEL_PARALLEL_ATTRIBUTE_DEFAULTS = {"tensor_model_parallel": False, "partition_dim": -1, "partition_stride": 1}


def param_is_not_tensor_parallel_duplicate(param):
    return (hasattr(param, "tensor_model_parallel") and param.tensor_model_parallel) or \
        ps.get_tensor_model_parallel_rank() == 0


def set_tensor_model_parallel_attributes(tensor, is_parallel, dim, stride):
    setattr(tensor, "tensor_model_parallel", is_parallel)
    setattr(tensor, "partition_dim", dim)
    setattr(tensor, "partition_stride", stride)


def set_defaults_if_not_set_tensor_model_parallel_attributes(tensor):
    for k, v in _MODEL_PARALLEL_ATTRIBUTE_DEFAULTS.items():
        if not hasattr(tensor, k):
            setattr(tensor, k, v)


def copy_tensor_model_parallel_attributes(destination, source):
    for k in _MODEL_PARALLEL_ATTRIBUTE_DEFAULTS:
        if hasattr(source, k):
            setattr(destination, k, getattr(source, k))


def _initialize_affine_weight(weight, output_size, input_size, per_partition_size, partition_dim,
                              init_method, stride=1, return_master_weight=False, params_dtype=torch.float32,
                              use_cpu_initialization=True):
    """Initialise the FULL weight identically on every rank (seeded), keep this rank's slice:
    results are independent of the TP degree (so TP runs match single-GPU runs).

    ``use_cpu_initialization``: the fp32 master is generated on the host (torch's CPU generator,
    bit-identical across machines); otherwise on the weight's device when that is a GPU (its seeded
    device generator — no host-memory copy of the full matrix, which for a 50k x 8k embedding is
    1.6 GB per rank)."""
    set_tensor_model_parallel_attributes(weight, True, partition_dim, stride)
    dev = weight.device if (not use_cpu_initialization and weight.device.type == "cuda") else torch.device("cpu")
    master = torch.empty(output_size, input_size, dtype=torch.float32, requires_grad=False, device=dev)
    init_method(master)
    master = master.to(params_dtype)
    per_stride = divide(per_partition_size, stride)
    chunks = torch.split(master, per_stride, dim=partition_dim)
    rank = ps.get_tensor_model_parallel_rank()
    ws = ps.get_tensor_model_parallel_world_size()
    mine = chunks[rank::ws]
    with torch.no_grad():
        weight.copy_(torch.cat(mine, dim=partition_dim))
    return master if return_master_weight else None


def _accumulate_main_grad(weight, dy2, x2, in_fp16=False):
    """weight.main_grad += dy2^T x2 without materialising a separate dW: fp32 accumulation (the
    GEMM's fp32 output with beta = 1) unless ``in_fp16`` (``accumulation_in_fp16``: main_grad kept
    in the activation dtype, accumulated there)."""
    mg = weight.main_grad
    if in_fp16 or mg.dtype != torch.float32:
        if mg.dtype == torch.float32:
            raise RuntimeError("accumulation_in_fp16 needs a 16-bit main_grad buffer")
        mg.addmm_(dy2.t().to(mg.dtype), x2.to(mg.dtype))
        return
    fops.accumulate_main_grad(mg, dy2, x2)


class LinearWithGradAccumulationAndAsyncCommunication(torch.autograd.Function):
    """y = x W^T (+ b) for a tensor-parallel shard, with the backward overlap described above."""

    @staticmethod
    def forward(ctx, x, weight, bias, gradient_accumulation_fusion, async_grad_allreduce, sequence_parallel,
                accumulation_in_fp16=False):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        ctx.flags = (gradient_accumulation_fusion, async_grad_allreduce, sequence_parallel)
        ctx.in_fp16 = bool(accumulation_in_fp16)
        total = _gather_seq(x) if sequence_parallel else x
        return fops.fused_dense(total, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        fusion, async_ar, sp = ctx.flags
        total = _gather_seq(x) if sp else x
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        t2 = total.reshape(-1, total.shape[-1])
        from ...ops import gemm as G

        dx = G.dgrad(dy2, weight).view(*dy.shape[:-1], weight.shape[1])
        handle, out = None, dx
        tp_group = ps.get_tensor_model_parallel_group()
        if ps.get_tensor_model_parallel_world_size() > 1:
            if sp:
                out = torch.empty((dx.shape[0] // ps.get_tensor_model_parallel_world_size(),) + tuple(dx.shape[1:]),
                                  dtype=dx.dtype, device=dx.device)
                handle = dist.reduce_scatter_tensor(out, dx.contiguous(), group=tp_group, async_op=True)
            elif async_ar:
                handle = dist.all_reduce(dx, group=tp_group, async_op=True)
        # weight gradient while the input-gradient collective is in flight
        if fusion and hasattr(weight, "main_grad") and weight.main_grad is not None:
            _accumulate_main_grad(weight, dy2, t2, ctx.in_fp16)
            if getattr(weight, "_apex_main_flat", None) is not None:
                # main_grad owned by apex DDP (fp32_main_grad): its hook must still see this
                # parameter become ready -> a placeholder gradient it drops
                dw = fops.main_grad_placeholder(weight)
            else:
                dw = None
        else:
            dw = fops._wgrad(dy2, t2, param=weight) if dy2.is_cuda else dy2.t().mm(t2)
        db = dy2.sum(0) if ctx.has_bias else None
        if handle is not None:
            handle.wait()
        return out, dw, db, None, None, None, None


def _gather_seq(x):
    ws = ps.get_tensor_model_parallel_world_size()
    if ws == 1:
        return x
    x = x.contiguous()
    out = torch.empty((ws * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x, group=ps.get_tensor_model_parallel_group())
    return out


def linear_with_grad_accumulation_and_async_allreduce(x, weight, bias, gradient_accumulation_fusion,
                                                      async_grad_allreduce, sequence_parallel_enabled,
                                                      accumulation_in_fp16=False):
    return LinearWithGradAccumulationAndAsyncCommunication.apply(x, weight, bias, gradient_accumulation_fusion,
                                                                 async_grad_allreduce, sequence_parallel_enabled,
                                                                 accumulation_in_fp16)


class VocabParallelEmbedding(nn.Module):
    """Embedding with the vocabulary split across the TP group; out-of-range ids produce 0
    locally and the all-reduce assembles the full lookup."""

    def __init__(self, num_embeddings, embedding_dim, init_method=nn.init.xavier_normal_, *,
                 params_dtype=torch.float32, use_cpu_initialization=False, device=None):
        super().__init__()
        self.num_embeddings = num_embeddings
        self.embedding_dim = embedding_dim
        self.tensor_model_parallel_size = ps.get_tensor_model_parallel_world_size()
        self.vocab_start_index, self.vocab_end_index = VocabUtility.vocab_range_from_global_vocab_size(
            num_embeddings, ps.get_tensor_model_parallel_rank(), self.tensor_model_parallel_size)
        self.num_embeddings_per_partition = self.vocab_end_index - self.vocab_start_index
        self.weight = Parameter(torch.empty(self.num_embeddings_per_partition, embedding_dim,
                                            dtype=params_dtype, device=device))
        _initialize_affine_weight(self.weight, num_embeddings, embedding_dim, self.num_embeddings_per_partition,
                                  0, init_method, params_dtype=params_dtype,
                                  use_cpu_initialization=use_cpu_initialization)

    def forward(self, input_):
        if self.tensor_model_parallel_size > 1:
            mask = (input_ < self.vocab_start_index) | (input_ >= self.vocab_end_index)
            local = input_.clone() - self.vocab_start_index
            local[mask] = 0
        else:
            local = input_
        out = F.embedding(local, self.weight)
        if self.tensor_model_parallel_size > 1:
            out = out.masked_fill(mask.unsqueeze(-1), 0.0)
        return reduce_from_tensor_model_parallel_region(out)


class ColumnParallelLinear(nn.Module):
    """Y = X A + b with A split by columns: A = [A_1 ... A_p]; rank i computes X A_i."""

    def __init__(self, input_size, output_size, bias=True, gather_output=True, init_method=nn.init.xavier_normal_,
                 stride=1, keep_master_weight_for_test=False, skip_bias_add=False, *,
                 no_async_tensor_model_parallel_allreduce=False, params_dtype=torch.float32,
                 use_cpu_initialization=False, gradient_accumulation_fusion=False,
                 accumulation_in_fp16=False, sequence_parallel_enabled=False, device=None):
        super().__init__()
        self.input_size = input_size
        self.output_size = output_size
        self.gather_output = gather_output
        ws = ps.get_tensor_model_parallel_world_size()
        self.output_size_per_partition = divide(output_size, ws)
        self.skip_bias_add = skip_bias_add
        self.sequence_parallel_enabled = sequence_parallel_enabled
        self.gradient_accumulation_fusion = gradient_accumulation_fusion
        self.accumulation_in_fp16 = accumulation_in_fp16
        # async dX all-reduce only where a backward all-reduce exists (TP > 1, no sequence parallel)
        self.async_tensor_model_parallel_allreduce = (not no_async_tensor_model_parallel_allreduce and ws > 1
                                                      and not sequence_parallel_enabled)
        self.weight = Parameter(torch.empty(self.output_size_per_partition, input_size, dtype=params_dtype,
                                            device=device))
        self.master_weight = _initialize_affine_weight(self.weight, output_size, input_size,
                                                       self.output_size_per_partition, 0, init_method, stride,
                                                       keep_master_weight_for_test, params_dtype,
                                                       use_cpu_initialization)
        if bias:
            self.bias = Parameter(torch.zeros(self.output_size_per_partition, dtype=params_dtype, device=device))
            set_tensor_model_parallel_attributes(self.bias, True, 0, stride)
        else:
            self.register_parameter("bias", None)

    def forward(self, input_):
        bias = self.bias if not self.skip_bias_add else None
        if self.async_tensor_model_parallel_allreduce or self.sequence_parallel_enabled or \
                self.gradient_accumulation_fusion:
            # the fused Function all-reduces (or reduce-scatters) dX itself only when async
            # all-reduce or sequence parallelism is on; with fusion alone the input goes through the
            # identity-forward / all-reduce-backward region first (Megatron's column-parallel rule)
            x = input_ if (self.async_tensor_model_parallel_allreduce or self.sequence_parallel_enabled) \
                else copy_to_tensor_model_parallel_region(input_)
            out = linear_with_grad_accumulation_and_async_allreduce(
                x, self.weight, bias, self.gradient_accumulation_fusion,
                self.async_tensor_model_parallel_allreduce, self.sequence_parallel_enabled,
                self.accumulation_in_fp16)
        else:
            out = fops.fused_dense(copy_to_tensor_model_parallel_region(input_), self.weight, bias)
        if self.gather_output:
            assert not self.sequence_parallel_enabled
            out = gather_from_tensor_model_parallel_region(out)
        return out, (self.bias if self.skip_bias_add else None)


class RowParallelLinear(nn.Module):
    """Y = X A + b with A split by rows (X split by columns); partial outputs all-reduced."""

    def __init__(self, input_size, output_size, bias=True, input_is_parallel=False,
                 init_method=nn.init.xavier_normal_, stride=1, keep_master_weight_for_test=False,
                 skip_bias_add=False, *, params_dtype=torch.float32, use_cpu_initialization=False,
                 gradient_accumulation_fusion=False, accumulation_in_fp16=False,
                 sequence_parallel_enabled=False, device=None):
        super().__init__()
        self.input_size = input_size
        self.output_size = output_size
        self.input_is_parallel = input_is_parallel
        ws = ps.get_tensor_model_parallel_world_size()
        self.input_size_per_partition = divide(input_size, ws)
        self.skip_bias_add = skip_bias_add
        self.sequence_parallel_enabled = sequence_parallel_enabled
        self.gradient_accumulation_fusion = gradient_accumulation_fusion
        self.accumulation_in_fp16 = accumulation_in_fp16
        if sequence_parallel_enabled and not input_is_parallel:
            raise RuntimeError("To enable `sequence_parallel_enabled`, `input_is_parallel` must be `True`")
        self.weight = Parameter(torch.empty(output_size, self.input_size_per_partition, dtype=params_dtype,
                                            device=device))
        self.master_weight = _initialize_affine_weight(self.weight, output_size, input_size,
                                                       self.input_size_per_partition, 1, init_method, stride,
                                                       keep_master_weight_for_test, params_dtype,
                                                       use_cpu_initialization)
        if bias:
            self.bias = Parameter(torch.zeros(output_size, dtype=params_dtype, device=device))
            setattr(self.bias, "sequence_parallel_enabled", sequence_parallel_enabled)
        else:
            self.register_parameter("bias", None)

    def forward(self, input_):
        x = input_ if self.input_is_parallel else scatter_to_tensor_model_parallel_region(input_)
        if self.gradient_accumulation_fusion:
            partial = linear_with_grad_accumulation_and_async_allreduce(x, self.weight, None, True, False, False,
                                                                        self.accumulation_in_fp16)
        else:
            partial = fops.fused_dense(x, self.weight, None)
        if self.sequence_parallel_enabled:
            out = reduce_scatter_to_sequence_parallel_region(partial)
        else:
            out = reduce_from_tensor_model_parallel_region(partial)
        if self.skip_bias_add:
            return out, self.bias
        return (out + self.bias if self.bias is not None else out), None
