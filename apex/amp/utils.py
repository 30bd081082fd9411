"""dtype-generic helpers for the amp cast engine (R-06).

The reference compared ``x.type()`` strings against 'HalfTensor'/'FloatTensor'
(apex/amp/utils.py:8-68); here every check is on ``torch.dtype`` and the low
precision type is configurable (fp16 or bf16) through ``set_low_dtype``.
Casts apply only to tensors on an accelerator device (CUDA/HIP), exactly like the
reference's ``maybe_half``/``maybe_float`` which left CPU tensors alone;
``set_cast_devices`` widens that set (tests use it to exercise the engine on CPU).
"""
from __future__ import annotations

import functools
import itertools

import torch

_LOW = [torch.float16]
_DEVICES = {"cuda"}


def set_low_dtype(dtype):
    assert dtype in (torch.float16, torch.bfloat16)
    _LOW[0] = dtype


def low_dtype():
    return _LOW[0]


def set_cast_devices(devices):
    _DEVICES.clear()
    _DEVICES.update(devices)


def is_nested(x):
    return isinstance(x, (tuple, list))


def is_fp_tensor(x):
    if is_nested(x):
        return all(is_fp_tensor(y) for y in x)
    return isinstance(x, torch.Tensor) and x.is_floating_point()


def should_cache(x):
    if is_nested(x):
        return all(should_cache(y) for y in x)
    return isinstance(x, torch.nn.Parameter) and x.dtype == torch.float32


def collect_fp_tensor_types(args, kwargs):
    types = set()

    def collect(x):
        if is_nested(x):
            for y in x:
                collect(y)
        elif isinstance(x, torch.Tensor) and x.is_floating_point():
            types.add(x.dtype)

    for x in itertools.chain(args, kwargs.values()):
        if is_fp_tensor(x):
            collect(x)
    return types


def _castable(x):
    return x.device.type in _DEVICES


def maybe_half(x, name="", verbose=False):
    """Cast an fp32 accelerator tensor to the low-precision dtype (else passthrough)."""
    if is_nested(x):
        return type(x)([maybe_half(y, name, verbose) for y in x])
    if not _castable(x) or x.dtype == _LOW[0] or not x.is_floating_point():
        return x
    if verbose:
        print("Float->{} ({})".format("Half" if _LOW[0] == torch.float16 else "BFloat16", name))
    return x.to(_LOW[0])


def maybe_float(x, name="", verbose=False):
    if is_nested(x):
        return type(x)([maybe_float(y, name, verbose) for y in x])
    if not _castable(x) or x.dtype == torch.float32 or not x.is_floating_point():
        return x
    if verbose:
        print("{}->Float ({})".format("Half" if x.dtype == torch.float16 else "BFloat16", name))
    return x.float()


def casted_args(cast_fn, args, kwargs):
    """Returns cast ``args``; mutates ``kwargs`` in place (reference contract)."""
    new_args = [cast_fn(x) if is_fp_tensor(x) else x for x in args]
    for k in kwargs:
        if is_fp_tensor(kwargs[k]):
            kwargs[k] = cast_fn(kwargs[k])
    return new_args


def cached_cast(cast_fn, x, cache):
    """Per-iteration cast cache keyed by the fp32 Parameter (fixes the reference's
    nested-branch bug at apex/amp/utils.py:86, which dropped cast_fn/cache)."""
    if is_nested(x):
        return type(x)([cached_cast(cast_fn, y, cache) for y in x])
    hit = cache.get(x)
    if hit is not None:
        if x.requires_grad != hit.requires_grad:
            hit.requires_grad_(x.requires_grad)
        return hit
    casted = cast_fn(x)
    cache[x] = casted
    return casted


def verbosify(cast_fn, fn_name, verbose):
    if verbose:
        return functools.partial(cast_fn, name=fn_name, verbose=verbose)
    return cast_fn


def as_inplace(fns):
    for x in fns:
        yield x + "_"


def has_func(mod, fn):
    if isinstance(mod, dict):
        return fn in mod
    return hasattr(mod, fn)


def get_func(mod, fn):
    if isinstance(mod, dict):
        return mod[fn]
    return getattr(mod, fn)


def set_func(mod, fn, new_fn):
    if isinstance(mod, dict):
        mod[fn] = new_fn
    else:
        setattr(mod, fn, new_fn)


def set_func_save(handle, mod, fn, new_fn):
    cur_fn = get_func(mod, fn)
    handle._save_func(mod, fn, cur_fn)
    set_func(mod, fn, new_fn)


def flat_low_precision_weights(weights, verbose=False, name=""):
    """Cast a list of fp32 RNN weights into ONE contiguous low-precision buffer.

    Each returned weight is a view at a running offset of a fresh flat buffer, filled
    with an autograd-tracked ``copy_`` from its fp32 source, so (a) the RNN kernel
    sees a single contiguous chunk (no per-call re-flatten / warning) and (b) the
    weight gradients flow back into the fp32 params. Replaces the reference's
    data_ptr-offset aliasing (apex/amp/utils.py:154-193).
    """
    total = sum(w.numel() for w in weights)
    flat = weights[0].new_empty((total,), dtype=_LOW[0])
    out, off = [], 0
    for w in weights:
        n = w.numel()
        v = flat[off:off + n].view_as(w)
        v.copy_(w)
        if verbose:
            print("Float->Half ({})".format(name))
        out.append(v)
        off += n
    return out
