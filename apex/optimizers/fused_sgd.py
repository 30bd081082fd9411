"""FusedSGD (NS-02): momentum / nesterov / weight-decay SGD in one HIP launch per group.

API follows apex.optimizers.FusedSGD:
``FusedSGD(params, lr, momentum=0., dampening=0., weight_decay=0., nesterov=False,
wd_after_momentum=False, materialize_master_grads=True, set_grad_none=False)``.
"""
from __future__ import annotations

import torch

from ..multi_tensor_apply import ops as mt_ops
from ._base import FusedOptimizerBase


class FusedSGD(FusedOptimizerBase):
    def __init__(self, params, lr=0.01, momentum=0.0, dampening=0.0, weight_decay=0.0,
                 nesterov=False, wd_after_momentum=False, materialize_master_grads=True,
                 set_grad_none=False):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if momentum < 0.0:
            raise ValueError(f"Invalid momentum value: {momentum}")
        if weight_decay < 0.0:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov)
        super().__init__(params, defaults, set_grad_none)
        self.wd_after_momentum = wd_after_momentum
        self.materialize_master_grads = materialize_master_grads
        self._first_run_flags = {}  # (group, dtype partition) -> int32[1] device flag

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        scale_t, scale_f = self._grad_scale_args()
        for gi, group in enumerate(self.param_groups):
            gs, ps, models = self._group_tensors(gi, group)
            if not gs:
                continue
            first_run = False
            moms = []
            for p in ps:
                st = self.state[p]
                if "momentum_buffer" not in st:
                    st["momentum_buffer"] = torch.zeros_like(p, dtype=torch.float32)
                    first_run = True
                moms.append(st["momentum_buffer"])
            lists = [gs, ps, moms] + ([models] if models is not None else [])
            if self._native(gs):
                # the first-run momentum init (buf = g, not (1-dampening) g) is keyed off a device
                # flag that only a step the loss scaler did NOT skip clears (a host flag
                # was used up by an overflow-skipped first step)
                for key, sub in self._split_by_dtype(lists):
                    flag = self._first_run_flags.get((gi, key))
                    if first_run or flag is None:
                        flag = self._first_run_flags[(gi, key)] = torch.full(
                            (1,), int(first_run), dtype=torch.int32, device=gs[0].device)
                    self._plan(("sgd", gi, key), sub).sgd(
                        float(group["lr"]), float(group["momentum"]), float(group["dampening"]),
                        float(group["weight_decay"]), bool(group["nesterov"]), first_run,
                        self.wd_after_momentum, scale_f, scale_t, self._amp_noop,
                        flag if self._amp_noop is not None else None)
            else:
                mt_ops.multi_tensor_sgd(0, self._amp_noop, lists, group["weight_decay"],
                                        group["momentum"], group["dampening"], group["lr"],
                                        group["nesterov"], first_run, self.wd_after_momentum,
                                        scale_t if scale_t is not None else scale_f)
        return loss

    def load_state_dict(self, state_dict):
        # the loaded momentum buffers are the state now: a first-run flag left at 1 by an
        # overflow-skipped first step would make the next step treat them as absent (buf = g)
        super().load_state_dict(state_dict)
        self._first_run_flags = {}
