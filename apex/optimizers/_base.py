"""Shared machinery for the fused optimizers (NS-02).

MI355X-first design points:
  * one MTPlan per param group, built once and re-validated by pointer in C++;
  * amp O2 "fused master" mode: the kernel reads the low-precision MODEL grads
    directly, multiplies by the device-resident inverse loss scale, updates the
    fp32 MASTER params and writes the low-precision model copy in the same pass
    (no materialised fp32 master grads, no separate master->model copy kernel);
  * overflow skip is decided on the device (``noop`` flag), so a training step
    never synchronises with the host.
"""
from __future__ import annotations

import torch
from torch.optim import Optimizer

from .. import _ext
from ..multi_tensor_apply import PlanHolder


def grad_of(p):
    """The gradient an optimizer should apply for ``p``: its fp32 ``main_grad`` (apex DDP
    fp32_main_grad mode; micro-batch gradients accumulated in fp32) or ``p.grad``."""
    mg = getattr(p, "main_grad", None)
    return mg if mg is not None else p.grad


class FusedOptimizerBase(Optimizer):
    def __init__(self, params, defaults, set_grad_none=True):
        super().__init__(params, defaults)
        self.set_grad_none = set_grad_none
        # amp integration (set by apex.amp when it owns this optimizer)
        self._amp_model_params = None    # list[list[Tensor]] per group (model copies)
        self._amp_grad_scale = None      # fp32 [1] device tensor: 1/loss_scale
        self._amp_noop = None            # int32 [1] device tensor: skip flag
        self._plans = {}
        # device step counters, key = (group index, ...) -> int32 [1]; advanced by the kernels
        # only when the step is not skipped. Not part of self.state: state_dict() publishes them
        # as param_group["step"] and load_state_dict() re-seeds them from it.
        self._dev_steps = {}

    def _device_step(self, key, group, device):
        t = self._dev_steps.get(key)
        if t is None or t.device != device:
            t = self._dev_steps[key] = torch.full((1,), int(group.get("step", 0)), dtype=torch.int32,
                                                  device=device)
        return t

    def _sync_steps_to_groups(self):
        for gi, group in enumerate(self.param_groups):
            vals = [int(t.item()) for k, t in self._dev_steps.items() if k[0] == gi]
            if vals:
                group["step"] = max(vals)

    def state_dict(self):
        self._sync_steps_to_groups()  # one host read per group; checkpointing only
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._dev_steps = {}
        self._plans = {}

    # ------------------------------------------------------------------
    def _plan(self, key, lists):
        h = self._plans.get(key)
        if h is None:
            h = self._plans[key] = PlanHolder()
        return h.get(lists)

    def _group_tensors(self, gi, group):
        """Returns (grads, params, model_copies or None) for group gi. A parameter's gradient is
        its fp32 ``main_grad`` when it has one (apex DDP fp32_main_grad mode), else ``.grad``."""
        params = [p for p in group["params"]]
        if self._amp_model_params is not None:
            models = self._amp_model_params[gi]
            sel = [(grad_of(m), p, m) for p, m in zip(params, models) if grad_of(m) is not None]
            if not sel:
                return [], [], []
            g, p, m = zip(*sel)
            return list(g), list(p), list(m)
        sel = [(grad_of(p), p) for p in params if grad_of(p) is not None]
        if not sel:
            return [], [], None
        g, p = zip(*sel)
        return list(g), list(p), None

    def zero_grad(self, set_to_none: bool | None = None):
        set_none = self.set_grad_none if set_to_none is None else set_to_none
        groups = self._amp_model_params if self._amp_model_params is not None else \
            [g["params"] for g in self.param_groups]
        # fp32 main_grad buffers (apex DDP fp32_main_grad): one fill per flat buffer
        main_flats = {}
        for ps in groups:
            for p in ps:
                f = getattr(p, "_apex_main_flat", None)
                if f is not None and getattr(p, "main_grad", None) is not None:
                    main_flats[id(f)] = f
                    p.grad = None
        for f in main_flats.values():
            f.zero_()
        # grads that are views of an apex DDP bucket buffer: one fill per buffer instead of one
        # launch per parameter, when every parameter of that buffer belongs to this optimizer
        flats, members = {}, {}
        for ps in groups:
            for p in ps:
                f = getattr(p, "_apex_bucket_flat", None)
                if p.grad is not None and f is not None and getattr(p, "_apex_grad_is_bucket_view", False):
                    flats[id(f)] = f
                    members[id(f)] = members.get(id(f), 0) + 1
        whole = {k for k, f in flats.items() if members[k] == getattr(f, "_apex_nparams", -1)}
        if set_none:
            # release the bucket views instead of zero-filling the buffers: the next backward's
            # fused producers then write each gradient straight into its slot
            # (apex.parallel.grad_target) and the rest are copied in by DDP, so no parameter pays
            # an accumulate kernel; DDP zero-fills the slots of parameters that get no gradient
            for ps in groups:
                for p in ps:
                    if p.grad is not None and id(getattr(p, "_apex_bucket_flat", None)) in whole:
                        p.grad = None
        else:
            for k in whole:
                flats[k].zero_()
        for ps in groups:
            for p in ps:
                if p.grad is None:
                    continue
                if whole and id(getattr(p, "_apex_bucket_flat", None)) in whole:
                    continue
                if set_none and not getattr(p, "_apex_grad_is_bucket_view", False):
                    p.grad = None
                else:
                    if p.grad.grad_fn is not None:
                        p.grad.detach_()
                    else:
                        p.grad.requires_grad_(False)
                    p.grad.zero_()

    @staticmethod
    def _split_by_dtype(lists):
        """Partition parallel tensor lists so every partition has ONE dtype per list (a plan's
        requirement). Groups mixing dtypes — e.g. amp O2 with fp32 BatchNorm next to bf16
        convs — become one launch per dtype combination. Returns [(dtype_key, lists)]."""
        parts = {}
        for i in range(len(lists[0])):
            parts.setdefault(tuple(l[i].dtype for l in lists), []).append(i)
        if len(parts) == 1:
            return [(next(iter(parts)), lists)]
        return [(k, [[l[i] for i in idx] for l in lists]) for k, idx in parts.items()]

    def _native(self, tensors):
        return len(tensors) > 0 and _ext.use_native(tensors[0])

    def _grad_scale_args(self):
        """(scale_tensor_or_None, scale_float)."""
        if self._amp_grad_scale is not None:
            return self._amp_grad_scale, 1.0
        return None, 1.0
