"""Loss-scaling context managers.

* ``amp.scale_loss(loss, optimizers, loss_id=0, ...)`` — new-style API (NS-01).
* ``AmpHandle`` / ``NoOpHandle`` — the reference's handle (R-03,
  apex/amp/handle.py:9-114): per-process cast cache, default scaler,
  ``scale_loss(loss, optimizer)``, ``wrap_optimizer``, ``_deactivate``.
"""
from __future__ import annotations

import contextlib
import logging
import warnings

import torch

from .. import _ext
from ..optimizers._base import FusedOptimizerBase
from ._amp_state import _amp_state, maybe_print
from .scaler import LossScaler


def _model_grads(optimizer):
    from ..optimizers._base import grad_of

    stash = getattr(optimizer, "_amp_stash", None)
    if stash is not None and stash.master_weights:
        return [grad_of(p) for ps in stash.model_params for p in ps if grad_of(p) is not None]
    return [grad_of(p) for g in optimizer.param_groups for p in g["params"] if grad_of(p) is not None]


@contextlib.contextmanager
def scale_loss(loss, optimizers, loss_id=0, model=None, delay_unscale=False,
               delay_overflow_check=False):
    """Yield ``loss * loss_scale``; on exit unscale grads / arm the optimizers.

    Fused apex optimizers receive the device inverse-scale and overflow flag and do
    the unscale inside their update kernel (no extra pass over the grads, no host
    sync). Other optimizers get one multi-tensor unscale(+copy to fp32 masters)
    launch and a single host read of the overflow flag (the reference behaviour).
    """
    props = _amp_state.opt_properties
    if props is None or not props.enabled:
        yield loss
        return
    if isinstance(optimizers, torch.optim.Optimizer) or hasattr(optimizers, "param_groups"):
        optimizers = [optimizers]
    scaler = _amp_state.loss_scalers[loss_id]
    scaler._ensure(loss.device)
    if not (scaler.dynamic or scaler._host_scale != 1.0) and not any(
            getattr(o, "_amp_stash", None) is not None and o._amp_stash.master_weights
            for o in optimizers):
        # scale 1, nothing to unscale or copy: fp32-equivalent fast path
        yield loss.float() if props.opt_level != "O3" else loss
        return
    yield scaler.scale_loss_value(loss)
    if delay_unscale:
        return
    for opt in optimizers:
        stash = getattr(opt, "_amp_stash", None)
        if stash is None:
            raise RuntimeError("Invoked 'with amp.scale_loss`, but internal Amp state has not been "
                               "initialized for this optimizer (pass it to amp.initialize).")
        if stash.fused:
            opt._amp_grad_scale = scaler.inv_scale_tensor
            if scaler.dynamic:
                opt._amp_noop = scaler.overflow_buf
                # LAMB's global-norm pass doubles as the overflow check; others need one pass
                from ..optimizers.fused_lamb import FusedLAMB
                if not isinstance(opt, FusedLAMB):
                    scaler.check_overflow(_model_grads(opt))
                scaler._device_skip_pending = True
            continue
        # ---- non-fused optimizer: unscale into masters (or in place) + host decision
        scaler.clear_overflow_state()
        if stash.master_weights:
            from ..optimizers._base import grad_of

            models = [m for m in stash.half_models if grad_of(m) is not None]
            masters = [ms for m, ms in zip(stash.half_models, stash.half_masters) if grad_of(m) is not None]
            for ms, m in zip(masters, models):
                if ms.grad is None:
                    ms.grad = torch.empty_like(ms)
            scaler.unscale([grad_of(m) for m in models], [ms.grad for ms in masters])
            fp32 = [p.grad for g in opt.param_groups for p in g["params"]
                    if p.grad is not None and all(p is not ms for ms in stash.half_masters)]
            if fp32:
                scaler.unscale(fp32, fp32)
        else:
            grads = _model_grads(opt)
            by_dt = {}
            for g in grads:
                by_dt.setdefault(g.dtype, []).append(g)
            for gl in by_dt.values():
                scaler.unscale(gl, gl)
        should_skip = scaler.update_scale_host()
        if should_skip:
            _skip_next_step(opt, scaler)


def _skip_next_step(optimizer, scaler):
    opt_step = optimizer.step

    def skip_step(closure=None):
        if closure is not None:
            raise RuntimeError("Currently, Amp does not support closure use with optimizers.")
        maybe_print(("Gradient overflow.  Skipping step, loss scaler {} reducing loss scale to {}")
                    .format(0, scaler.loss_scale()))
        stash = optimizer._amp_stash
        if stash.master_weights:
            for ms in stash.half_masters:
                ms.grad = None
        optimizer.step = opt_step

    optimizer.step = skip_step


# ---------------------------------------------------------------------------
# Reference handle (apex v0.1 amp.init API)
# ---------------------------------------------------------------------------
class AmpHandle:
    def __init__(self, enable_caching=True, verbose=False, loss_scale="dynamic"):
        self._enable_caching = enable_caching
        self._verbose = verbose
        self._cache = dict()
        self._default_scaler = LossScaler(loss_scale)
        self._is_active = True
        self._all_wrappers = []

    def is_active(self):
        return self._is_active

    @contextlib.contextmanager
    def _disable_casts(self):
        self._is_active = False
        try:
            yield
        finally:
            self._is_active = True

    def wrap_optimizer(self, optimizer, num_loss=1):
        from .opt import OptimWrapper

        self._default_scaler = None
        return OptimWrapper(optimizer, self, num_loss)

    @contextlib.contextmanager
    def scale_loss(self, loss, optimizer):
        if not self.is_active():
            yield loss
            return
        if self._default_scaler is None:
            raise RuntimeError("After calling `handle.wrap_optimizer()`, you must explicitly "
                               "use `optimizer.scale_loss(loss)`.")

        # TODO(reference parity): warn if the unscaled loss is backpropagated
        def warning_wrapper():
            warnings.warn("You called .backward() on the unscaled loss inside a scale_loss block. "
                          "This is almost certainly an error.", stacklevel=2)
            orig_backward()

        orig_backward = loss.backward
        loss.backward = warning_wrapper
        loss_scale = self._default_scaler.loss_scale()
        try:
            yield loss * loss_scale
        finally:
            loss.backward = orig_backward
        should_skip = self._default_scaler.unscale_and_update(optimizer.param_groups, loss_scale)
        if should_skip:
            optimizer_step = optimizer.step

            def skip_step(closure=None):
                logging.info("Gradient overflow, skipping update")
                optimizer.step = optimizer_step

            optimizer.step = skip_step
        self._clear_cache()

    def _clear_cache(self):
        self._cache.clear()

    # Experimental support for saving / restoring uncasted versions of functions
    def _save_func(self, mod, fn, func):
        self._all_wrappers.append((mod, fn, func))

    def _deactivate(self):
        for mod, fn, func in self._all_wrappers:
            setattr(mod, fn, func)
        self._all_wrappers = []
        self._is_active = False
        from . import rnn_compat

        rnn_compat.restore()

    @property
    def has_cache(self):
        return self._enable_caching

    @property
    def cache(self):
        return self._cache

    def remove_cache(self, param):
        if self.has_cache and param in self.cache:
            del self.cache[param]

    @property
    def verbose(self):
        return self._verbose


class NoOpHandle:
    def is_active(self):
        return False

    @contextlib.contextmanager
    def _disable_casts(self):
        yield

    def wrap_optimizer(self, optimizer, num_loss=1):
        from .opt import OptimWrapper

        return OptimWrapper(optimizer, self, num_loss)

    @contextlib.contextmanager
    def scale_loss(self, loss, optimizer):
        yield loss

    @property
    def has_cache(self):
        return False

    @property
    def verbose(self):
        return False

    def _clear_cache(self):
        pass

    def _deactivate(self):
        pass
