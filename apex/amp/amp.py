"""Reference amp API (R-01, R-02): ``init`` + decorator / registry forms.

Placeholder during bring-up; the cast-policy engine lands in apex/amp/wrap.py.
"""
from __future__ import annotations

import functools

_DECORATOR_HANDLE = None
_USER_CAST_REGISTRY = set()
_USER_PROMOTE_REGISTRY = set()


def half_function(fn):
    return fn


def bfloat16_function(fn):
    return fn


def float_function(fn):
    return fn


def promote_function(fn):
    return fn


def register_half_function(module, name):
    if not hasattr(module, name):
        raise ValueError("No function named {} in module {}.".format(name, module))
    _USER_CAST_REGISTRY.add((module, name, "half"))


def register_bfloat16_function(module, name):
    register_half_function(module, name)


def register_float_function(module, name):
    if not hasattr(module, name):
        raise ValueError("No function named {} in module {}.".format(name, module))
    _USER_CAST_REGISTRY.add((module, name, "float"))


def register_promote_function(module, name):
    if not hasattr(module, name):
        raise ValueError("No function named {} in module {}.".format(name, module))
    _USER_PROMOTE_REGISTRY.add((module, name))


def init(enabled=True, enable_caching=True, verbose=False, allow_banned=False, loss_scale="dynamic",
         half_dtype=None):
    raise NotImplementedError("amp.init cast engine: pending")
