"""Model / optimizer preparation for ``amp.initialize`` (NS-01).

O2 semantics follow ``network_to_half`` + ``FP16_Optimizer``
(apex/fp16_utils/fp16util.py:21-41, apex/fp16_utils/fp16_optimizer.py:105-175):
BatchNorm stays fp32, every low-precision param gets an fp32 master that is swapped
into the optimizer's param_groups. For apex's fused optimizers the masters are
updated by the fused kernel straight from the low-precision model grads (see
apex/optimizers/_base.py); for any other optimizer the unscale+copy (K-01/K-02)
and master->model copy run as single multi-tensor launches around ``step``.
"""
from __future__ import annotations

import functools
import types

import torch
from torch import nn

from .. import _ext
from ..multi_tensor_apply import get_plan
from ..multi_tensor_apply import ops as mt_ops
from ..optimizers._base import FusedOptimizerBase
from ._amp_state import _amp_state, maybe_print, warn_or_err
from .scaler import LossScaler


def _is_float(t):
    return isinstance(t, torch.Tensor) and t.is_floating_point()


def applier(value, fn):
    if isinstance(value, torch.Tensor):
        return fn(value)
    if isinstance(value, str):
        return value
    if isinstance(value, dict):
        return {k: applier(v, fn) for k, v in value.items()}
    if isinstance(value, tuple) and hasattr(value, "_fields"):
        return type(value)(*[applier(v, fn) for v in value])
    if isinstance(value, (list, tuple)):
        return type(value)(applier(v, fn) for v in value)
    return value


def to_type(dtype, t):
    if isinstance(t, torch.Tensor) and t.is_floating_point():
        return t.to(dtype)
    return t


_BN_TYPES = (nn.modules.batchnorm._BatchNorm,)


def convert_module(module, dtype):
    for p in module.parameters(recurse=False):
        if p is not None and p.is_floating_point():
            p.data = p.data.to(dtype)
            if p._grad is not None:
                p._grad.data = p._grad.data.to(dtype)
    for name, b in module.named_buffers(recurse=False):
        if b is not None and b.is_floating_point():
            setattr(module, name, b.to(dtype))


def convert_network(network, dtype, keep_batchnorm_fp32=True):
    """Cast a network to ``dtype`` keeping BatchNorm (incl. SyncBatchNorm) in fp32."""
    for m in network.modules():
        if keep_batchnorm_fp32 and isinstance(m, _BN_TYPES) and m.affine:
            continue
        if getattr(m, "_amp_keep_fp32", False):
            continue
        convert_module(m, dtype)
    return network


def check_models(models):
    for model in models:
        parallel = (torch.nn.parallel.DistributedDataParallel, torch.nn.parallel.DataParallel)
        if isinstance(model, parallel):
            raise RuntimeError("Incoming model is an instance of torch.nn.parallel."
                               "DistributedDataParallel. Parallel wrappers should only be applied "
                               "to the model(s) AFTER the model(s) have been returned from "
                               "amp.initialize.")


def check_optimizers(optimizers):
    for o in optimizers:
        if getattr(o, "_amp_stash", None) is not None:
            raise RuntimeError("An optimizer was passed to amp.initialize twice.")


class _AmpStash:
    pass


def _process_optimizer(optimizer, properties):
    stash = optimizer._amp_stash = _AmpStash()
    stash.fused = isinstance(optimizer, FusedOptimizerBase)
    stash.master_weights = bool(properties.master_weights)
    stash.model_params = []    # per group: list of model params (low precision or fp32)
    stash.fp32_from_half = []  # per group: masters for the low-precision ones
    stash.half_models = []     # flat list: low-precision model params (non-fused path)
    stash.half_masters = []    # flat list: their fp32 masters
    if stash.master_weights:
        for gi, group in enumerate(optimizer.param_groups):
            models, new_params = [], []
            for i, p in enumerate(group["params"]):
                models.append(p)
                if p.requires_grad and p.dtype in (torch.float16, torch.bfloat16):
                    master = p.detach().clone().float()
                    master.requires_grad = True
                    master = nn.Parameter(master)
                    new_params.append(master)
                    if p in optimizer.state:
                        optimizer.state[master] = optimizer.state.pop(p)
                    stash.half_models.append(p)
                    stash.half_masters.append(master)
                elif p.dtype == torch.float32:
                    new_params.append(p)
                else:
                    raise TypeError("Optimizer's parameters must be float32, float16 or bfloat16. "
                                    "Received {}".format(p.type()))
            group["params"] = new_params
            stash.model_params.append(models)
        if stash.fused:
            optimizer._amp_model_params = stash.model_params
    _patch_step(optimizer)
    return optimizer


def _patch_step(optimizer):
    old_step = optimizer.step
    stash = optimizer._amp_stash

    def new_step(self, closure=None):
        if closure is not None:
            raise RuntimeError("Currently, Amp does not support closure use with optimizers.")
        retval = old_step()
        if stash.master_weights and not stash.fused and stash.half_models:
            # master -> model copy (K-02), one launch
            if _ext.use_native(stash.half_masters[0]):
                get_plan([stash.half_masters, stash.half_models]).scale(None, 1.0, None)
            else:
                for m, p in zip(stash.half_masters, stash.half_models):
                    p.data.copy_(m.data)
        for scaler in _amp_state.loss_scalers:
            scaler._post_step_pending = True
        _post_step_scalers(self)
        if getattr(_amp_state, "fp8", False):
            from .. import fp8 as _fp8

            _fp8.step()  # fold this step's amaxes into the scales; drop the cached fp8 weights
        return retval

    optimizer.step = types.MethodType(new_step, optimizer)

    old_zero = optimizer.zero_grad

    def new_zero_grad(self, set_to_none=None):
        if stash.master_weights and not stash.fused:
            for models in stash.model_params:
                for p in models:
                    if p.grad is not None:
                        if getattr(p, "_apex_grad_is_bucket_view", False):
                            p.grad.zero_()
                        else:
                            p.grad = None
            for group in self.param_groups:
                for p in group["params"]:
                    p.grad = None
            return None
        if set_to_none is None:
            return old_zero()
        return old_zero(set_to_none=set_to_none)

    optimizer.zero_grad = types.MethodType(new_zero_grad, optimizer)


def _post_step_scalers(optimizer):
    """After a (possibly device-skipped) step: update dynamic scales on the device."""
    stash = optimizer._amp_stash
    for scaler in _amp_state.loss_scalers:
        if getattr(scaler, "_device_skip_pending", False):
            scaler.update_scale()
            scaler.clear_overflow_state()
            scaler._device_skip_pending = False
    if stash.fused:
        optimizer._amp_noop = None


def _initialize(models, optimizers, properties, num_losses=1, cast_model_outputs=None):
    optimizers_was_list = isinstance(optimizers, list)
    if optimizers is None:
        optimizers = []
    elif not isinstance(optimizers, list):
        optimizers = [optimizers]
    models_was_list = isinstance(models, list)
    if not models_was_list:
        models = [models]
    check_models(models)
    check_optimizers(optimizers)

    if properties.cast_model_type is not None and properties.cast_model_type != torch.float32:
        for model in models:
            convert_network(model, properties.cast_model_type,
                            keep_batchnorm_fp32=bool(properties.keep_batchnorm_fp32))
        input_caster = functools.partial(to_type, properties.cast_model_type)
        out_t = cast_model_outputs if cast_model_outputs is not None else torch.float32
        output_caster = functools.partial(to_type, out_t)
        for model in models:
            def patch_forward(old_fwd):
                @functools.wraps(old_fwd)
                def new_fwd(*args, **kwargs):
                    output = old_fwd(*applier(args, input_caster), **applier(kwargs, input_caster))
                    return applier(output, output_caster)
                return new_fwd
            model.forward = patch_forward(model.forward)
    elif properties.cast_model_type == torch.float32:
        for model in models:
            model.float()

    for i, opt in enumerate(optimizers):
        optimizers[i] = _process_optimizer(opt, properties)

    _amp_state.loss_scalers = []
    for _ in range(num_losses):
        _amp_state.loss_scalers.append(LossScaler(properties.loss_scale,
                                                  min_loss_scale=_amp_state.min_loss_scale,
                                                  max_loss_scale=_amp_state.max_loss_scale))
    _amp_state.optimizers = optimizers

    if properties.patch_torch_functions:
        from .amp import init as _legacy_init

        handle = _legacy_init(enabled=True, loss_scale=properties.loss_scale, verbose=(_amp_state.verbosity == 2),
                              half_dtype=properties.half_dtype)
        _amp_state.handle = handle
        if cast_model_outputs is not None:
            out_caster = functools.partial(to_type, cast_model_outputs)
            for model in models:
                def patch_forward(old_fwd):
                    @functools.wraps(old_fwd)
                    def new_fwd(*args, **kwargs):
                        return applier(old_fwd(*args, **kwargs), out_caster)
                    return new_fwd
                model.forward = patch_forward(model.forward)

    if optimizers_was_list:
        out_opts = optimizers
    elif len(optimizers) == 1:
        out_opts = optimizers[0]
    else:
        out_opts = None
    out_models = models if models_was_list else models[0]
    if out_opts is None and not optimizers_was_list:
        return out_models
    return out_models, out_opts
