"""FusedAdam / AdamW (NS-02): one HIP launch per param group per step.

API follows apex.optimizers.FusedAdam (later apex releases):
``FusedAdam(params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8,
adam_w_mode=True, weight_decay=0., amsgrad=False, set_grad_none=True, capturable=False,
master_weights=False, max_grad_norm=0.)``.

* ``master_weights``: fp32 master copies of 16-bit parameters live in the optimizer; the kernel
  reads the 16-bit grads, updates the fp32 masters and writes the 16-bit parameters in the same
  pass (the amp O2 "fused master" mode, without amp);
* ``capturable``: the native step never synchronises with the host (device step counter, device
  overflow flag), so it is always graph-capturable; the flag only checks that every parameter is
  on the GPU, as upstream's capturable mode requires;
* legacy ``step(closure, grads, output_params, scale, grad_norms)``: explicit gradient tensors
  instead of ``p.grad``, 16-bit ``output_params`` written with the updated fp32 parameters, grads
  divided by ``scale``, and with ``max_grad_norm > 0`` clipped by ``grad_norms`` (the global norm
  of the scaled grads): combined scale = scale * max(1, (norm / scale + 1e-6) / max_grad_norm).
"""

from __future__ import annotations

import torch

from ..multi_tensor_apply import ops as mt_ops
from ._base import FusedOptimizerBase


class FusedAdam(FusedOptimizerBase):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8,
                 adam_w_mode=True, weight_decay=0.0, amsgrad=False, set_grad_none=True,
                 capturable=False, master_weights=False, max_grad_norm=0.0):
        if amsgrad:
            raise RuntimeError("FusedAdam does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                        weight_decay=weight_decay, max_grad_norm=max_grad_norm)
        super().__init__(params, defaults, set_grad_none)
        self.adam_w_mode = 1 if adam_w_mode else 0
        self.capturable = capturable
        self.master_weights = master_weights
        if capturable:
            for g in self.param_groups:
                for p in g["params"]:
                    if not p.is_cuda:
                        raise RuntimeError("FusedAdam(capturable=True) needs every parameter on the GPU")

    def _master(self, p):
        """fp32 master of a 16-bit parameter, kept in the optimizer state (checkpointed with it)."""
        st = self.state[p]
        m = st.get("master_param")
        if m is None:
            m = st["master_param"] = p.detach().clone().float()
        return m

    def _explicit_tensors(self, gi, group, grads, output_params):
        """(grads, params, models) from the legacy explicit-list arguments (per group, or flat
        lists for a single group)."""
        ps = list(group["params"])
        g = grads[gi] if (grads and isinstance(grads[0], (list, tuple))) else grads
        o = None
        if output_params is not None:
            o = output_params[gi] if (output_params and isinstance(output_params[0], (list, tuple))) \
                else output_params
        sel = [i for i in range(len(ps)) if g[i] is not None]
        if not sel:
            return [], [], None
        return [g[i] for i in sel], [ps[i] for i in sel], ([o[i] for i in sel] if o is not None else None)

    @torch.no_grad()
    def step(self, closure=None, grads=None, output_params=None, scale=None, grad_norms=None):
        loss = closure() if closure is not None else None
        scale_t, scale_f = self._grad_scale_args()
        if scale is not None:  # legacy apex signature: grads are divided by `scale`
            scale_f = 1.0 / float(scale)
        for gi, group in enumerate(self.param_groups):
            if grads is not None:
                gs, ps, models = self._explicit_tensors(gi, group, grads, output_params)
            else:
                gs, ps, models = self._group_tensors(gi, group)
            if not gs:
                continue
            if self.master_weights and models is None and self._amp_model_params is None:
                # 16-bit params: the fp32 master is updated, the param is the written model copy
                if any(p.dtype != torch.float32 for p in ps):
                    models = list(ps)
                    ps = [self._master(p) if p.dtype != torch.float32 else p for p in ps]
            gscale = scale_f
            mgn = float(group.get("max_grad_norm", 0.0))
            if grad_norms is not None and mgn > 0:
                norm = grad_norms[gi] if isinstance(grad_norms, (list, tuple)) else grad_norms
                s0 = float(scale) if scale is not None else 1.0
                clip = (float(norm) / s0 + 1e-6) / mgn
                if clip > 1:
                    gscale = scale_f / clip
            b1, b2 = group["betas"]
            states = []
            owners = models if (models is not None and self.master_weights) else ps
            for p, own in zip(ps, owners):
                st = self.state[own]  # state keyed by the user's parameter (master_weights too)
                if "exp_avg" not in st:
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
                        gscale, scale_t, self._amp_noop, step_t, bool(group["bias_correction"]))
            else:
                if self._amp_noop is not None and int(self._amp_noop.item()) != 0:
                    continue
                group["step"] = group.get("step", 0) + 1
                mt_ops.multi_tensor_adam(0, self._amp_noop, lists, group["lr"], b1, b2,
                                         group["eps"], group["step"], self.adam_w_mode,
                                         group["bias_correction"], group["weight_decay"],
                                         scale_t if scale_t is not None else gscale)
        return loss
