"""FusedLAMB (NS-02) — layer-wise adaptive large-batch optimizer, HIP fused.

Semantics follow apex's FusedLAMB (later apex releases; not in the v0.1
reference, listed as north-star in BASELINE.json):
  global grad norm over ALL groups -> clip divisor max(1, ||g|| / max_grad_norm)
  m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2 ; u = m^/(sqrt(v^)+eps) + wd p
  p -= lr * (||p|| / ||u||) * u     (trust ratio when wd != 0 or use_nvlamb)

Device pipeline per step (csrc/multi_tensor.hip): one l2norm over all grads
(+overflow flag) -> per group: prep (device step++, bias corrections), stage1
(moments, per-chunk norms of p and of the update u), per-tensor norm reduce, stage2
(recompute u from the new moments, apply + bf16 model copy). No host synchronisation,
no parameter-sized scratch buffer; the device step counters are published as
``param_group["step"]`` by state_dict() and re-seeded from it by load_state_dict(), so a
checkpoint loaded with ``map_location="cpu"`` resumes on the GPU.
"""
from __future__ import annotations

import torch

from ..multi_tensor_apply import ops as mt_ops
from ..utils import prof
from ._base import FusedOptimizerBase


class FusedLAMB(FusedOptimizerBase):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-6,
                 weight_decay=0.01, amsgrad=False, adam_w_mode=True, grad_averaging=True,
                 set_grad_none=True, max_grad_norm=1.0, use_nvlamb=False):
        if amsgrad:
            raise RuntimeError("FusedLAMB does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                        weight_decay=weight_decay, grad_averaging=grad_averaging,
                        max_grad_norm=max_grad_norm)
        super().__init__(params, defaults, set_grad_none)
        self.adam_w_mode = 1 if adam_w_mode else 0
        self.use_nvlamb = use_nvlamb
        self._gnorm = None

    def _state_for(self, p):
        st = self.state[p]
        if len(st) == 0:
            st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32)
            st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32)
        return st

    def _group_step(self, key, group, device):
        return self._device_step(key, group, device)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        per_group = [self._group_tensors(gi, g) for gi, g in enumerate(self.param_groups)]
        all_grads = [g for (gs, _, _) in per_group for g in gs]
        if not all_grads:
            return loss
        with prof.range("apex.optim.FusedLAMB.step"):
            if self._native(all_grads):
                self._step_native(per_group, all_grads)
            else:
                self._step_reference(per_group, all_grads)
        return loss

    # ------------------------------------------------------------------
    def _step_native(self, per_group, all_grads):
        dev = all_grads[0].device
        scale_t, scale_f = self._grad_scale_args()
        noop = self._amp_noop
        # one global norm over every group's grads (also raises the overflow flag)
        by_dtype = {}
        for g in all_grads:
            by_dtype.setdefault(g.dtype, []).append(g)
        sq = None
        for dt, gl in by_dtype.items():
            gn, _ = self._plan(("gnorm", dt), [gl]).l2norm(0, False, scale_t, scale_f, noop)
            sq = gn * gn if sq is None else sq + gn * gn
        gnorm = sq.sqrt() if len(by_dtype) > 1 else gn
        self._gnorm = gnorm
        for gi, (group, (gs, ps, models)) in enumerate(zip(self.param_groups, per_group)):
            if not gs:
                continue
            b1, b2 = group["betas"]
            states = [self._state_for(p) for p in ps]
            lists = [gs, ps, [s["exp_avg"] for s in states], [s["exp_avg_sq"] for s in states]]
            if models is not None:
                lists.append(models)
            for key, sub in self._split_by_dtype(lists):
                # the prep kernel advances its step counter once per launch: one counter per
                # dtype partition keeps every partition at the group's true step
                step_t = self._group_step((gi, key) if len(sub[0]) != len(gs) else (gi,), group, dev)
                self._plan(("lamb", gi, key), sub).lamb(
                    float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                    float(group["weight_decay"]), float(group["max_grad_norm"]),
                    self.adam_w_mode == 1, bool(group["bias_correction"]),
                    bool(group["grad_averaging"]), bool(self.use_nvlamb), scale_f, scale_t, noop, None,
                    step_t, gnorm)

    def _step_reference(self, per_group, all_grads):
        scale = float(self._amp_grad_scale.item()) if self._amp_grad_scale is not None else 1.0
        if self._amp_noop is not None and int(self._amp_noop.item()) != 0:
            return
        gnorm = torch.stack([g.float().norm() for g in all_grads]).pow(2).sum().sqrt() * scale
        if not bool(torch.isfinite(gnorm)) and self._amp_noop is not None:
            self._amp_noop.fill_(1)
            return
        self._gnorm = gnorm
        for gi, (group, (gs, ps, models)) in enumerate(zip(self.param_groups, per_group)):
            if not gs:
                continue
            b1, b2 = group["betas"]
            states = [self._state_for(p) for p in ps]
            step_t = self._group_step((gi,), group, gs[0].device)
            step_t += 1
            mt_ops.lamb_reference(gs, ps, [s["exp_avg"] for s in states],
                                  [s["exp_avg_sq"] for s in states], group["lr"], b1, b2,
                                  group["eps"], int(step_t.item()), group["bias_correction"],
                                  group["weight_decay"], group["grad_averaging"], self.adam_w_mode,
                                  float(gnorm), group["max_grad_norm"], self.use_nvlamb,
                                  grad_scale=scale, copies=models)
