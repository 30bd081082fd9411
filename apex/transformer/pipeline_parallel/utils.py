"""Microbatch bookkeeping and loss helpers for pipeline / data parallel training."""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import parallel_state as ps
from ..microbatches import build_num_microbatches_calculator

_GLOBAL_NUM_MICROBATCHES_CALCULATOR = None


def setup_microbatch_calculator(rank, rampup_batch_size, global_batch_size, micro_batch_size, data_parallel_size):
    global _GLOBAL_NUM_MICROBATCHES_CALCULATOR
    _GLOBAL_NUM_MICROBATCHES_CALCULATOR = build_num_microbatches_calculator(
        rank, rampup_batch_size, global_batch_size, micro_batch_size, data_parallel_size)


def _reconfigure_microbatch_calculator(rank, rampup_batch_size, global_batch_size, micro_batch_size,
                                       data_parallel_size):
    setup_microbatch_calculator(rank, rampup_batch_size, global_batch_size, micro_batch_size, data_parallel_size)


def get_micro_batch_size():
    return _GLOBAL_NUM_MICROBATCHES_CALCULATOR.micro_batch_size


def get_num_microbatches():
    if _GLOBAL_NUM_MICROBATCHES_CALCULATOR is None:
        return 1
    return _GLOBAL_NUM_MICROBATCHES_CALCULATOR.get()


def get_current_global_batch_size():
    return _GLOBAL_NUM_MICROBATCHES_CALCULATOR.get_current_global_batch_size()


def update_num_microbatches(consumed_samples, consistency_check=True):
    _GLOBAL_NUM_MICROBATCHES_CALCULATOR.update(consumed_samples, consistency_check)


def get_kth_microbatch(batch, k):
    if batch is None:
        return None
    mbs = get_micro_batch_size()
    return [x[k * mbs:(k + 1) * mbs] for x in batch]


def average_losses_across_data_parallel_group(losses):
    averaged = torch.cat([l.clone().detach().view(1) for l in losses])
    dist.all_reduce(averaged, group=ps.get_data_parallel_group())
    return averaged / dist.get_world_size(group=ps.get_data_parallel_group())


def listify_model(model):
    return model if isinstance(model, list) else [model]


def unwrap_model(model, module_instances=(torch.nn.parallel.DistributedDataParallel,)):
    return_list = True
    if not isinstance(model, list):
        model = [model]
        return_list = False
    out = []
    for m in model:
        while isinstance(m, module_instances) or hasattr(m, "module") and type(m).__name__ in (
                "DistributedDataParallel",):
            m = m.module
        out.append(m)
    return out if return_list else out[0]


def calc_params_l2_norm(model, bf16=False):
    norms = [p.detach().float().norm() for m in listify_model(model) for p in m.parameters()]
    sq = torch.stack(norms).pow(2).sum() if norms else torch.zeros(())
    if dist.is_initialized():
        dist.all_reduce(sq, group=ps.get_model_parallel_group())
    return sq.sqrt().item()
