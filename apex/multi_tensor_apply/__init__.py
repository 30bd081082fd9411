"""Multi-tensor apply (K-01/K-02/K-07 host side).

``MTPlan`` (C++ in csrc/bindings.cpp) is a device-resident chunk table for N
parallel tensor lists; every fused op is ONE launch over every chunk of every
tensor. Plans are cached by tensor identity and re-validated by raw pointer in
C++, so a steady-state training step performs no metadata upload.

Public API mirrors later apex releases:
    multi_tensor_applier(op, noop_flag_buffer, tensor_lists, *args)
with ops from ``apex.multi_tensor_apply.ops`` (``multi_tensor_scale``,
``multi_tensor_axpby``, ``multi_tensor_l2norm``, ``multi_tensor_sgd``,
``multi_tensor_adam``, ``multi_tensor_lamb``).
Reference: the removed ``apex_C.scale_check_overflow`` (apex/amp/scaler.py:3) and
"Carl's fused kernel" TODO (apex/fp16_utils/fp16_optimizer.py:10).
"""
from __future__ import annotations

from collections import OrderedDict

import torch

from .. import _ext

DEFAULT_CHUNK = 32768

_plan_cache: "OrderedDict[tuple, object]" = OrderedDict()
_PLAN_CACHE_MAX = 64


def get_plan(tensor_lists, chunk_size: int = DEFAULT_CHUNK):
    """Return a (cached) MTPlan for ``tensor_lists`` (lists of device tensors)."""
    C = _ext.require()
    key = (chunk_size,) + tuple(tuple(id(t) for t in lst) for lst in tensor_lists)
    plan = _plan_cache.get(key)
    if plan is not None and plan.matches(tensor_lists):
        _plan_cache.move_to_end(key)
        return plan
    plan = C.MTPlan([list(lst) for lst in tensor_lists], chunk_size)
    _plan_cache[key] = plan
    if len(_plan_cache) > _PLAN_CACHE_MAX:
        _plan_cache.popitem(last=False)
    return plan


class PlanHolder:
    """Per-owner plan (optimizers keep one per param group; no global cache churn)."""

    def __init__(self, chunk_size: int = DEFAULT_CHUNK):
        self.chunk_size = chunk_size
        self.plan = None

    def get(self, tensor_lists):
        if self.plan is None or not self.plan.matches(tensor_lists):
            self.plan = _ext.require().MTPlan([list(l) for l in tensor_lists], self.chunk_size)
        return self.plan


class MultiTensorApply:
    available = True
    warned = False

    def __init__(self, chunk_size: int = DEFAULT_CHUNK):
        self.chunk_size = chunk_size

    def __call__(self, op, noop_flag_buffer, tensor_lists, *args):
        return op(self.chunk_size, noop_flag_buffer, tensor_lists, *args)


multi_tensor_applier = MultiTensorApply(DEFAULT_CHUNK)

from . import ops  # noqa: E402,F401
