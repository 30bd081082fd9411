"""LARC optimizer wrapper (R-18, K-07).

Reference (apex/parallel/LARC.py:40-97): per-param adaptive lr
``trust * ||p|| / (||g|| + ||p||*wd + eps)`` (clip mode: ``min(adaptive/lr, 1)``),
weight decay absorbed into the grad, restored after ``step``. The reference ran two
host-synchronised ``torch.norm`` per parameter; here all norms and the grad rescale
are 5 launches per param group with no host sync (csrc/multi_tensor.hip mt_larc).
"""
from __future__ import annotations

import torch

from .. import _ext
from ..multi_tensor_apply import PlanHolder


class LARC:
    def __init__(self, optimizer, trust_coefficient=0.02, clip=True, eps=1e-8):
        self.param_groups = optimizer.param_groups
        self.optim = optimizer
        self.trust_coefficient = trust_coefficient
        self.eps = eps
        self.clip = clip
        self._plans = {}

    def __getstate__(self):
        return self.optim.__getstate__()

    def __setstate__(self, state):
        self.optim.__setstate__(state)

    def __repr__(self):
        return self.optim.__repr__()

    @property
    def state(self):
        return self.optim.state

    def state_dict(self):
        return self.optim.state_dict()

    def load_state_dict(self, state_dict):
        self.optim.load_state_dict(state_dict)

    def zero_grad(self, *args, **kwargs):
        self.optim.zero_grad(*args, **kwargs)

    def add_param_group(self, param_group):
        self.optim.add_param_group(param_group)

    def _apply_group(self, gi, group, weight_decay):
        ps = [p for p in group["params"] if p.grad is not None]
        if not ps:
            return
        gs = [p.grad for p in ps]
        if _ext.use_native(gs[0]):
            by_dt = {}
            for g, p in zip(gs, ps):
                by_dt.setdefault((g.dtype, p.dtype), ([], []))
                by_dt[(g.dtype, p.dtype)][0].append(g)
                by_dt[(g.dtype, p.dtype)][1].append(p)
            for key, (gl, pl) in by_dt.items():
                h = self._plans.setdefault((gi, key), PlanHolder())
                h.get([gl, pl]).larc(self.trust_coefficient, self.eps, float(group["lr"]),
                                     float(weight_decay), bool(self.clip))
            return
        for p in ps:
            param_norm = torch.norm(p.data)
            grad_norm = torch.norm(p.grad.data)
            if param_norm != 0 and grad_norm != 0:
                adaptive_lr = self.trust_coefficient * param_norm / (
                    grad_norm + param_norm * weight_decay + self.eps)
                if self.clip:
                    adaptive_lr = min(adaptive_lr / group["lr"], 1)
                p.grad.data += weight_decay * p.data
                p.grad.data *= adaptive_lr

    def step(self, closure=None):
        with torch.no_grad():
            weight_decays = []
            for gi, group in enumerate(self.optim.param_groups):
                weight_decay = group.get("weight_decay", 0)
                weight_decays.append(weight_decay)
                group["weight_decay"] = 0
                self._apply_group(gi, group, weight_decay)
        try:
            return self.optim.step(closure) if closure is not None else self.optim.step()
        finally:
            for i, group in enumerate(self.optim.param_groups):
                group["weight_decay"] = weight_decays[i]
