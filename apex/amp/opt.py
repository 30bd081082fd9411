"""OptimWrapper (R-04): an optimizer with ``num_loss`` independently scaled losses.

Reference: apex/amp/opt.py:9-108. For ``loss_idx > 0`` the grads accumulated so far
are stashed and zeroed before backward, so each loss is unscaled with its own scale,
then the stash is added back. The stash/restore is a multi-tensor axpby on device.
Fixed vs reference: the loss-scaler state is included in ``state_dict``.
"""
from __future__ import annotations

import contextlib
import logging
import warnings

import torch

from .scaler import LossScaler


def iter_params(param_groups):
    for group in param_groups:
        for p in group["params"]:
            yield p


class OptimWrapper:
    def __init__(self, optimizer, amp_handle, num_loss):
        self._optimizer = optimizer
        self._amp_handle = amp_handle
        self._num_loss = num_loss
        self._loss_idx = 0
        self._skip_next = [False] * num_loss
        self._loss_scaler = [LossScaler("dynamic") for _ in range(num_loss)]

    @contextlib.contextmanager
    def scale_loss(self, loss):
        if not self._amp_handle.is_active():
            yield loss
            return
        loss_backward = loss.backward

        def warning_wrapper():
            warnings.warn("You called .backward() on the unscaled loss inside a scale_loss block. "
                          "This is almost certainly an error.", stacklevel=2)
            loss_backward()

        loss.backward = warning_wrapper
        cached_grads = []
        if self._loss_idx > 0:
            for p in iter_params(self._optimizer.param_groups):
                cached_grads.append(p.grad.detach().clone() if p.grad is not None else None)
            self._optimizer.zero_grad()
        loss_scale = self._cur_loss_scaler().loss_scale()
        try:
            yield loss * loss_scale
        finally:
            loss.backward = loss_backward
        self._skip_next[self._loss_idx] = self._cur_loss_scaler().unscale_and_update(
            self._optimizer.param_groups, loss_scale)
        self._loss_idx += 1
        if cached_grads:
            for p, cg in zip(iter_params(self._optimizer.param_groups), cached_grads):
                if cg is not None:
                    if p.grad is None:
                        p.grad = cg
                    else:
                        p.grad.data.add_(cg)

    def _cur_loss_scaler(self):
        assert 0 <= self._loss_idx < self._num_loss
        return self._loss_scaler[self._loss_idx]

    def step(self, closure=None):
        if not self._amp_handle.is_active():
            return self._optimizer.step(closure=closure)
        self._loss_idx = 0
        for p in iter_params(self._optimizer.param_groups):
            self._amp_handle.remove_cache(p)
        if closure is not None:
            raise NotImplementedError("The `closure` argument is unsupported by the amp optimizer wrapper.")
        if any(self._skip_next):
            logging.info("Gradient overflow, skipping update")
            self._skip_next = [False] * self._num_loss
            return None
        return self._optimizer.step()

    def __getattr__(self, attr):
        return getattr(self._optimizer, attr)

    def __getstate__(self):
        return self._optimizer.__getstate__()

    def __setstate__(self, state):
        return self._optimizer.__setstate__(state)

    def __repr__(self):
        return self._optimizer.__repr__()

    def state_dict(self):
        sd = self._optimizer.state_dict()
        sd["amp_loss_scalers"] = [s.state_dict() for s in self._loss_scaler]
        return sd

    def load_state_dict(self, state_dict):
        state_dict = dict(state_dict)
        scalers = state_dict.pop("amp_loss_scalers", None)
        if scalers is not None:
            for s, sd in zip(self._loss_scaler, scalers):
                s.load_state_dict(sd)
        return self._optimizer.load_state_dict(state_dict)

    def zero_grad(self, *args, **kwargs):
        return self._optimizer.zero_grad(*args, **kwargs)

    def add_param_group(self, param_group):
        return self._optimizer.add_param_group(param_group)
