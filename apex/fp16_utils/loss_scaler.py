"""Static / dynamic loss scalers for FP16_Optimizer (R-12).

Reference semantics (apex/fp16_utils/loss_scaler.py:10-132) preserved exactly:
  * DynamicLossScaler(init_scale=2**32, scale_factor=2., scale_window=1000);
  * on overflow: ``cur_scale = max(cur_scale / scale_factor, 1)``;
  * growth when ``(cur_iter - last_overflow_iter) % scale_window == 0`` — so the
    first growth happens at iteration 999;
  * ``has_overflow(params)`` — here ONE fused multi-tensor check per dtype over all
    grads (K-01) instead of a host-synchronising ``float(x.sum())`` per param; the
    result is read back once.
"""
from __future__ import annotations

import torch

from .. import _ext


def to_python_float(t):
    if hasattr(t, "item"):
        return t.item()
    return t[0]


def _grads_overflow(params) -> bool:
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return False
    if _ext.use_native(grads[0]):
        from ..multi_tensor_apply import get_plan

        flag = torch.zeros(1, dtype=torch.int32, device=grads[0].device)
        by_dt = {}
        for g in grads:
            by_dt.setdefault(g.dtype, []).append(g.contiguous() if not g.is_contiguous() else g)
        for gl in by_dt.values():
            get_plan([gl]).l2norm(0, False, None, 1.0, flag)
        return bool(flag.item())
    return any(DynamicLossScaler._has_inf_or_nan(g) for g in grads)


class LossScaler:
    """Static loss scale (``has_overflow`` is always False)."""

    def __init__(self, scale=1):
        self.cur_scale = scale

    def has_overflow(self, params):
        return False

    @staticmethod
    def _has_inf_or_nan(x):
        return False

    def update_scale(self, overflow):
        pass

    @property
    def loss_scale(self):
        return self.cur_scale

    def scale_gradient(self, module, grad_in, grad_out):
        return tuple(self.loss_scale * g for g in grad_in)

    def backward(self, loss):
        scaled_loss = loss * self.loss_scale
        scaled_loss.backward()

    def state_dict(self):
        return dict(cur_scale=self.cur_scale)

    def load_state_dict(self, sd):
        self.cur_scale = sd["cur_scale"]


class DynamicLossScaler:
    """Dynamic loss scale: back off on overflow, grow every ``scale_window`` clean iters."""

    def __init__(self, init_scale=2 ** 32, scale_factor=2.0, scale_window=1000):
        self.cur_scale = init_scale
        self.cur_iter = 0
        self.last_overflow_iter = -1
        self.scale_factor = scale_factor
        self.scale_window = scale_window

    def has_overflow(self, params):
        return _grads_overflow(params)

    @staticmethod
    def _has_inf_or_nan(x):
        try:
            cpu_sum = float(x.float().sum())
        except RuntimeError as instance:
            if "value cannot be converted" not in instance.args[0]:
                raise
            return True
        if cpu_sum == float("inf") or cpu_sum == -float("inf") or cpu_sum != cpu_sum:
            return True
        return False

    def update_scale(self, overflow):
        if overflow:
            self.cur_scale = max(self.cur_scale / self.scale_factor, 1)
            self.last_overflow_iter = self.cur_iter
        else:
            if (self.cur_iter - self.last_overflow_iter) % self.scale_window == 0:
                self.cur_scale *= self.scale_factor
        self.cur_iter += 1

    @property
    def loss_scale(self):
        return self.cur_scale

    def scale_gradient(self, module, grad_in, grad_out):
        return tuple(self.loss_scale * g for g in grad_in)

    def backward(self, loss):
        scaled_loss = loss * self.loss_scale
        scaled_loss.backward()

    def state_dict(self):
        return dict(cur_scale=self.cur_scale, cur_iter=self.cur_iter,
                    last_overflow_iter=self.last_overflow_iter, scale_factor=self.scale_factor,
                    scale_window=self.scale_window)

    def load_state_dict(self, sd):
        for k, v in sd.items():
            setattr(self, k, v)
