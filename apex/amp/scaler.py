"""amp loss scaling (R-09, K-01) with a device-resident scale.

Reference: apex/amp/scaler.py:20-60 — dynamic scaler with init 2**16, max 2**24,
growth window 2000, x2 / /2, no floor; ``unscale_and_update`` walked every param
with a host-synchronising ``float(grad.sum())`` (scaler.py:9).

Here the scale, its growth tracker and the overflow flag live on the device:
unscale+check of every grad is ONE multi-tensor launch and the scale update is a
1-thread kernel, so the hot path never waits on the host. Host reads happen only
where the API demands a Python bool (``unscale_and_update`` for non-fused
optimizers) or when the user asks for ``loss_scale()``.
"""
from __future__ import annotations

import torch

from .. import _ext
from ..multi_tensor_apply import get_plan
from ..multi_tensor_apply import ops as mt_ops


def scale_check_overflow(d_grads, scale):
    """Legacy per-tensor helper (reference scaler.py:6-18): returns True on inf/nan,
    otherwise scales ``d_grads`` in place by ``scale``."""
    if not bool(torch.isfinite(d_grads).all()):
        return True
    d_grads.mul_(scale)
    return False


class LossScaler:
    warned_no_fused_kernel = False
    warned_unscaling_non_fp32_grad = False
    has_fused_kernel = True

    def __init__(self, loss_scale="dynamic", init_scale=2.0 ** 16, scale_factor=2.0,
                 scale_window=2000, min_loss_scale=None, max_loss_scale=2.0 ** 24):
        self.dynamic = loss_scale == "dynamic"
        self._init = float(init_scale) if self.dynamic else float(loss_scale)
        self._scale_factor = float(scale_factor)
        self._scale_window = int(scale_window)
        self._min_loss_scale = min_loss_scale
        self._max_loss_scale = max_loss_scale
        self._device = None
        self._scale = None        # fp32 0-dim device tensor
        self._inv_scale = None    # fp32 0-dim device tensor (kept in sync lazily)
        self._tracker = None      # int32 [1]
        self._overflow = None     # int32 [1]
        self._host_scale = self._init
        self._unskipped = 0
        self._has_overflow = False

    # ------------------------------------------------------------------ state
    def _ensure(self, device):
        if self._scale is not None and self._device == device:
            return
        self._device = device
        self._scale = torch.full((), self._host_scale, dtype=torch.float32, device=device)
        self._inv_scale = torch.full((), 1.0 / self._host_scale, dtype=torch.float32, device=device)
        self._tracker = torch.full((1,), self._unskipped, dtype=torch.int32, device=device)
        self._overflow = torch.zeros(1, dtype=torch.int32, device=device)

    def loss_scale(self):
        if self._scale is None:
            return self._host_scale
        return float(self._scale.item())

    @property
    def scale_tensor(self):
        return self._scale

    @property
    def inv_scale_tensor(self):
        return self._inv_scale

    @property
    def overflow_buf(self):
        return self._overflow

    def scale_loss_value(self, loss):
        self._ensure(loss.device)
        return loss.float() * self._scale

    def clear_overflow_state(self):
        self._has_overflow = False
        if self._overflow is not None:
            self._overflow.zero_()

    # ------------------------------------------------------------- unscale ops
    def unscale(self, model_grads, master_grads, unused_scale=None, models_are_masters=False):
        """master = model * (1/scale) with overflow check (one launch)."""
        if not model_grads:
            return
        self._ensure(model_grads[0].device)
        if _ext.use_native(model_grads[0]):
            get_plan([model_grads, master_grads]).scale(self._inv_scale, 1.0, self._overflow)
        else:
            mt_ops.multi_tensor_scale(0, self._overflow, [model_grads, master_grads],
                                      1.0 / self.loss_scale())

    def check_overflow(self, grads):
        """Overflow check only (used ahead of fused optimizers that unscale in-kernel)."""
        if not grads:
            return
        self._ensure(grads[0].device)
        by_dt = {}
        for g in grads:
            by_dt.setdefault(g.dtype, []).append(g)
        for gl in by_dt.values():
            mt_ops.multi_tensor_l2norm(32768, self._overflow, [gl], False)

    def unscale_with_stashed(self, model_grads, stashed_master_grads, master_grads):
        """master = model/scale + stashed (gradient accumulation across losses)."""
        if not model_grads:
            return
        self._ensure(model_grads[0].device)
        inv = 1.0 / self.loss_scale()
        mt_ops.multi_tensor_axpby(32768, self._overflow,
                                  [model_grads, stashed_master_grads, master_grads], inv, 1.0, 0)

    def update_scale(self):
        """Device-side update; returns nothing (see ``update_scale_host`` for a bool)."""
        if self._scale is None:
            return
        if self.dynamic:
            mt_ops.update_scale_(self._scale, self._tracker, self._overflow, self._scale_factor,
                                 1.0 / self._scale_factor, self._scale_window,
                                 self._min_loss_scale or 0.0,
                                 self._max_loss_scale if self._max_loss_scale else float("inf"))
            torch.reciprocal(self._scale, out=self._inv_scale)

    def update_scale_host(self):
        """Reference-compatible update returning should_skip (one host read)."""
        if self._overflow is None:
            return False
        self._has_overflow = bool(self._overflow.item()) if self.dynamic else False
        self.update_scale()
        if self._has_overflow:
            self._unskipped = 0
        else:
            self._unskipped += 1
        return self._has_overflow

    # ------------------------------------------------- legacy (apex v0.1) API
    def unscale_and_update(self, param_groups, scale):
        """Reference API (apex/amp/scaler.py:32-55): unscale all grads in place by
        ``1/scale`` and update the scale; returns True when the step must be skipped."""
        grads = [p.grad for g in param_groups for p in g["params"] if p.grad is not None]
        if grads:
            self._ensure(grads[0].device)
            self._overflow.zero_()
            if _ext.use_native(grads[0]):
                by_dt = {}
                for g in grads:
                    by_dt.setdefault(g.dtype, []).append(g)
                for gl in by_dt.values():
                    get_plan([gl, gl]).scale(None, 1.0 / scale, self._overflow)
            else:
                mt_ops.multi_tensor_scale(0, self._overflow, [grads, grads], 1.0 / scale)
        should_skip = bool(self._overflow.item()) if self._overflow is not None else False
        if should_skip:
            self._host_scale = self.loss_scale() / self._scale_factor
            if self._min_loss_scale:
                self._host_scale = max(self._host_scale, self._min_loss_scale)
            self._unskipped = 0
        else:
            self._unskipped += 1
        if self._unskipped == self._scale_window and self.dynamic:
            self._host_scale = min(self._max_loss_scale, self.loss_scale() * self._scale_factor)
            self._unskipped = 0
        if self._scale is not None:
            self._scale.fill_(self._host_scale)
            self._inv_scale.fill_(1.0 / self._host_scale)
            self._tracker.fill_(self._unskipped)
        return should_skip

    # -------------------------------------------------------------- checkpoint
    def state_dict(self):
        return {"loss_scale": self.loss_scale(), "unskipped": int(self._tracker.item())
                if self._tracker is not None else self._unskipped}

    def load_state_dict(self, sd):
        self._host_scale = float(sd["loss_scale"])
        self._unskipped = int(sd.get("unskipped", 0))
        if self._scale is not None:
            self._scale.fill_(self._host_scale)
            self._inv_scale.fill_(1.0 / self._host_scale)
            self._tracker.fill_(self._unskipped)
