"""Reference amp API (R-01, R-02): ``init`` + decorator / registry forms.

``init()`` installs every cast hook in the reference's order (apex/amp/amp.py:57-163):
user cast registry, user promote registry, low/fp32 tables over F / torch / Tensor,
promotion (multi-arg and sequence), in-place fp32 ops erroring on low precision,
other in-place ops matching ``self``, RNNs and RNN cells, banned functions.
``handle._deactivate()`` restores every patched attribute.

MI355X additions: ``half_dtype=torch.bfloat16`` runs the whole policy in bf16.
"""
from __future__ import annotations

import functools
import itertools

import torch

from . import rnn_compat, utils, wrap
from .handle import AmpHandle, NoOpHandle
from .policy import FUNCTIONAL, TENSOR, TORCH

_DECORATOR_HANDLE = None
_USER_CAST_REGISTRY = []   # (module, name, cast_fn); list: modules need not be hashable
_USER_PROMOTE_REGISTRY = []


def _decorator_helper(orig_fn, cast_fn, wrap_fn):
    @functools.wraps(orig_fn)
    def wrapper(*args, **kwargs):
        handle = _DECORATOR_HANDLE
        if handle is None or not handle.is_active():
            return orig_fn(*args, **kwargs)
        inner = utils.verbosify(cast_fn, orig_fn.__name__, handle.verbose)
        return wrap_fn(orig_fn, inner, handle)(*args, **kwargs)

    return wrapper


def half_function(fn):
    return _decorator_helper(fn, utils.maybe_half,
                             functools.partial(wrap.make_cast_wrapper, try_caching=True))


bfloat16_function = half_function


def float_function(fn):
    return _decorator_helper(fn, utils.maybe_float,
                             functools.partial(wrap.make_cast_wrapper, try_caching=False))


def promote_function(fn):
    return _decorator_helper(fn, utils.maybe_float, wrap.make_promote_wrapper)


def _add(reg, entry):
    if not any(e[0] is entry[0] and e[1:] == entry[1:] for e in reg):
        reg.append(entry)


def _check(module, name):
    if not hasattr(module, name):
        raise ValueError("No function named {} in module {}.".format(name, module))


def register_half_function(module, name):
    _check(module, name)
    _add(_USER_CAST_REGISTRY, (module, name, utils.maybe_half))


register_bfloat16_function = register_half_function


def register_float_function(module, name):
    _check(module, name)
    _add(_USER_CAST_REGISTRY, (module, name, utils.maybe_float))


def register_promote_function(module, name):
    _check(module, name)
    _add(_USER_PROMOTE_REGISTRY, (module, name))


def init(enabled=True, enable_caching=True, verbose=False, allow_banned=False, loss_scale="dynamic",
         half_dtype=None):
    global _DECORATOR_HANDLE
    if not enabled:
        handle = NoOpHandle()
        _DECORATOR_HANDLE = handle
        return handle
    utils.set_low_dtype(half_dtype or torch.float16)
    handle = AmpHandle(enable_caching, verbose, loss_scale)

    # 0) user-registered casts, 0.5) user-registered promotions
    for mod, fn, cast_fn in list(_USER_CAST_REGISTRY):
        wrap.cached_cast(mod, fn, cast_fn, handle, cast_fn is utils.maybe_half, verbose)
    _USER_CAST_REGISTRY.clear()
    for mod, fn in list(_USER_PROMOTE_REGISTRY):
        wrap.promote(mod, fn, handle, verbose)
    _USER_PROMOTE_REGISTRY.clear()

    # 1) low-precision / fp32 tables
    for table, (cat, cast_fn) in itertools.product(
            (FUNCTIONAL, TORCH, TENSOR), (("low", utils.maybe_half), ("fp32", utils.maybe_float))):
        for fn in table[cat]:
            wrap.cached_cast(table["module"], fn, cast_fn, handle, cast_fn is utils.maybe_half, verbose)

    # 2) promotion on multi-arg and sequence ops
    for table in (TORCH, TENSOR):
        for fn in table["promote"]:
            wrap.promote(table["module"], fn, handle, verbose)
        for fn in table["sequence"]:
            wrap.sequence_promote(table["module"], fn, handle, verbose)

    # 3) in-place fp32 functions error on low-precision inputs
    for fn in utils.as_inplace(TORCH["fp32"]):
        wrap.err_if_any_half(TORCH["module"], fn, handle)
    # 3.5) in-place fp32 methods error when self is low precision
    for fn in utils.as_inplace(TENSOR["fp32"]):
        wrap.err_if_arg0_half(TENSOR["module"], fn, handle, verbose)
    # 4) other in-place methods cast their args to self's dtype
    for fn in utils.as_inplace(itertools.chain(TENSOR["low"], TENSOR["promote"])):
        wrap.promote_match_arg0(TENSOR["module"], fn, handle, verbose)

    # 5) RNNs + RNN cells run in low precision
    rnn_compat.whitelist_rnns(handle, verbose)
    rnn_compat.whitelist_rnn_cells(handle, verbose)

    # 6) banned functions
    for fn, err_msg in FUNCTIONAL["banned"]:
        if allow_banned:
            wrap.cached_cast(FUNCTIONAL["module"], fn, utils.maybe_float, handle, True, verbose)
        else:
            wrap.err_if_any_half(FUNCTIONAL["module"], fn, handle, err_msg)

    _DECORATOR_HANDLE = handle
    return handle
