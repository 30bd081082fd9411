"""FusedAdam / AdamW (NS-02): one HIP launch per param group per step.

API follows apex.optimizers.FusedAdam (later apex releases):
``FusedAdam(params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8,
adam_w_mode=True, weight_decay=0., amsgrad=False, set_grad_none=True)``.
"""
from __future__ import annotations

import torch

from ..multi_tensor_apply import ops as mt_ops
from ._base import FusedOptimizerBase


class FusedAdam(FusedOptimizerBase):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8,
                 adam_w_mode=True, weight_decay=0.0, amsgrad=False, set_grad_none=True,
                 capturable=False, master_weights=False):
        if amsgrad:
            raise RuntimeError("FusedAdam does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                        weight_decay=weight_decay)
        super().__init__(params, defaults, set_grad_none)
        self.adam_w_mode = 1 if adam_w_mode else 0

    @torch.no_grad()
    def step(self, closure=None, grads=None, output_params=None, scale=None, grad_norms=None):
        loss = closure() if closure is not None else None
        scale_t, scale_f = self._grad_scale_args()
        if scale is not None:  # legacy apex signature: grads are divided by `scale`
            scale_f = 1.0 / float(scale)
        for gi, group in enumerate(self.param_groups):
            gs, ps, models = self._group_tensors(gi, group)
            if not gs:
                continue
            b1, b2 = group["betas"]
            states = []
            for p in ps:
                st = self.state[p]
                if len(st) == 0:
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32)
                    st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32)
                states.append(st)
            lists = [gs, ps, [s["exp_avg"] for s in states], [s["exp_avg_sq"] for s in states]]
            if models is not None:
                lists.append(models)
            if self._native(gs):
                # the step count (and so the bias corrections) lives on the device and advances
                # only when the loss scaler did not skip the step (a host counter
                # kept counting overflow-skipped steps)
                for key, sub in self._split_by_dtype(lists):
                    step_t = self._device_step((gi, key), group, gs[0].device)
                    self._plan(("adam", gi, key), sub).adam(
                        float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                        float(group["weight_decay"]), 1.0, 1.0, self.adam_w_mode == 1,
                        scale_f, scale_t, self._amp_noop, step_t, bool(group["bias_correction"]))
            else:
                if self._amp_noop is not None and int(self._amp_noop.item()) != 0:
                    continue
                group["step"] = group.get("step", 0) + 1
                mt_ops.multi_tensor_adam(0, self._amp_noop, lists, group["lr"], b1, b2,
                                         group["eps"], group["step"], self.adam_w_mode,
                                         group["bias_correction"], group["weight_decay"],
                                         scale_t if scale_t is not None else scale_f)
        return loss
