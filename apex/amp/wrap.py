"""Cast-wrapper factories for the amp engine (R-05).

Same wrapper taxonomy as the reference (apex/amp/wrap.py:8-249) — cast-all with
per-iteration Parameter caching, widest-type promotion for multi-arg and sequence
ops, match-self for in-place methods, error-if-low-precision for in-place fp32
ops, RNN interposition — expressed on dtypes so fp16 and bf16 both work.
"""
from __future__ import annotations

import functools

import torch

from . import utils


def make_cast_wrapper(orig_fn, cast_fn, handle, try_caching=False):
    @functools.wraps(orig_fn)
    def wrapper(*args, **kwargs):
        if not handle.is_active():
            return orig_fn(*args, **kwargs)
        if try_caching and handle.has_cache:
            args = list(args)
            for i, a in enumerate(args):
                if utils.should_cache(a):
                    args[i] = utils.cached_cast(cast_fn, a, handle.cache)
            for k in kwargs:
                if utils.should_cache(kwargs[k]):
                    kwargs[k] = utils.cached_cast(cast_fn, kwargs[k], handle.cache)
        new_args = utils.casted_args(cast_fn, args, kwargs)
        return orig_fn(*new_args, **kwargs)

    return wrapper


def cached_cast(mod, fn, cast_fn, handle, try_caching=False, verbose=False):
    if not utils.has_func(mod, fn):
        return
    orig_fn = utils.get_func(mod, fn)
    cast_fn = utils.verbosify(cast_fn, fn, verbose)
    utils.set_func_save(handle, mod, fn, make_cast_wrapper(orig_fn, cast_fn, handle, try_caching))


def make_promote_wrapper(orig_fn, cast_fn, handle=None):
    @functools.wraps(orig_fn)
    def wrapper(*args, **kwargs):
        if handle is not None and not handle.is_active():
            return orig_fn(*args, **kwargs)
        types = utils.collect_fp_tensor_types(args, kwargs)
        if len(types) <= 1:
            return orig_fn(*args, **kwargs)
        if types == {utils.low_dtype(), torch.float32}:
            return orig_fn(*utils.casted_args(cast_fn, args, kwargs), **kwargs)
        raise NotImplementedError("Do not know how to handle these types to promote: {}".format(types))

    return wrapper


def promote(mod, fn, handle, verbose=False):
    if not utils.has_func(mod, fn):
        return
    orig_fn = utils.get_func(mod, fn)
    maybe_float = utils.verbosify(utils.maybe_float, fn, verbose)
    utils.set_func_save(handle, mod, fn, make_promote_wrapper(orig_fn, maybe_float, handle))


def sequence_promote(mod, fn, handle, verbose=False):
    if not utils.has_func(mod, fn):
        return
    orig_fn = utils.get_func(mod, fn)
    maybe_float = utils.verbosify(utils.maybe_float, fn, verbose)

    @functools.wraps(orig_fn)
    def wrapper(seq, *args, **kwargs):
        if not handle.is_active():
            return orig_fn(seq, *args, **kwargs)
        types = {x.dtype for x in seq if isinstance(x, torch.Tensor) and x.is_floating_point()}
        if types == {utils.low_dtype(), torch.float32}:
            return orig_fn(utils.casted_args(maybe_float, seq, {}), *args, **kwargs)
        return orig_fn(seq, *args, **kwargs)

    utils.set_func_save(handle, mod, fn, wrapper)


def promote_match_arg0(mod, fn, handle, verbose=False):
    if not utils.has_func(mod, fn):
        return
    orig_fn = utils.get_func(mod, fn)

    @functools.wraps(orig_fn)
    def wrapper(arg0, *args, **kwargs):
        if not handle.is_active() or not isinstance(arg0, torch.Tensor):
            return orig_fn(arg0, *args, **kwargs)
        if arg0.dtype == utils.low_dtype():
            cast_fn = utils.maybe_half
        elif arg0.dtype == torch.float32:
            cast_fn = utils.maybe_float
        else:
            return orig_fn(arg0, *args, **kwargs)
        cast_fn = utils.verbosify(cast_fn, fn, verbose)
        return orig_fn(arg0, *utils.casted_args(cast_fn, args, kwargs), **kwargs)

    utils.set_func_save(handle, mod, fn, wrapper)


def err_if_any_half(mod, fn, handle, custom_err_msg=None):
    if not utils.has_func(mod, fn):
        return
    orig_fn = utils.get_func(mod, fn)

    @functools.wraps(orig_fn)
    def wrapper(*args, **kwargs):
        if handle.is_active() and utils.low_dtype() in utils.collect_fp_tensor_types(args, kwargs):
            if custom_err_msg:
                raise NotImplementedError(custom_err_msg)
            raise NotImplementedError("Cannot call in-place function {} with fp16 arguments.".format(fn))
        return orig_fn(*args, **kwargs)

    utils.set_func_save(handle, mod, fn, wrapper)


def err_if_arg0_half(mod, fn, handle, verbose=False):
    if not utils.has_func(mod, fn):
        return
    orig_fn = utils.get_func(mod, fn)

    @functools.wraps(orig_fn)
    def wrapper(arg0, *args, **kwargs):
        if not handle.is_active() or not isinstance(arg0, torch.Tensor):
            return orig_fn(arg0, *args, **kwargs)
        if arg0.dtype == utils.low_dtype():
            raise NotImplementedError("Cannot call in-place method {} on fp16 Tensors.".format(fn))
        cast_fn = utils.verbosify(utils.maybe_float, fn, verbose)
        return orig_fn(arg0, *utils.casted_args(cast_fn, args, kwargs), **kwargs)

    utils.set_func_save(handle, mod, fn, wrapper)


def rnn_cast(shim, fn, handle, verbose=False):
    """Interpose on a full-sequence RNN entry of the ``_VF`` shim (``lstm``/``gru``/
    ``rnn_tanh``/``rnn_relu``): input, hidden state and all weights go to low
    precision, the weights as ONE contiguous buffer (utils.flat_low_precision_weights)."""
    orig_fn = utils.get_func(shim, fn)
    cast_fn = utils.verbosify(utils.maybe_half, fn, verbose)

    @functools.wraps(orig_fn)
    def wrapper(*args, **kwargs):
        if not handle.is_active():
            return orig_fn(*args, **kwargs)
        # torch signatures: (input, hx, params, has_biases, ...) or
        # (data, batch_sizes, hx, params, has_biases, ...) for packed sequences.
        params_idx = 2 if isinstance(args[3], bool) else 3
        new_args = []
        for i, a in enumerate(args):
            if i == params_idx:
                ws = list(a)
                if ws and all(w.dtype == torch.float32 for w in ws) and ws[0].device.type in utils._DEVICES:
                    new_args.append(utils.flat_low_precision_weights(ws, verbose, fn))
                else:
                    new_args.append([cast_fn(w) for w in ws])
            elif isinstance(a, (list, tuple)) and a and all(isinstance(t, torch.Tensor) for t in a):
                new_args.append(type(a)(cast_fn(t) if t.is_floating_point() else t for t in a))
            elif utils.is_fp_tensor(a):
                new_args.append(cast_fn(a))
            else:
                new_args.append(a)
        return orig_fn(*new_args, **kwargs)

    utils.set_func_save(handle, shim, fn, wrapper)


def disable_casts(mod, fn, handle):
    if not utils.has_func(mod, fn):
        return
    orig_fn = utils.get_func(mod, fn)

    @functools.wraps(orig_fn)
    def wrapper(*args, **kwargs):
        with handle._disable_casts():
            return orig_fn(*args, **kwargs)

    utils.set_func_save(handle, mod, fn, wrapper)
