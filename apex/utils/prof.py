"""Profiler ranges. On ROCm builds ``torch.cuda.nvtx`` is backed by roctx, so ranges show up
in ``rocprofv3 --marker-trace`` timelines; they are also emitted as
``torch.profiler.record_function`` scopes for the PyTorch profiler. Disabled (zero cost
beyond one attribute check) unless ``APEX_PROF_RANGES=1`` or ``enable(True)``."""
from __future__ import annotations

import contextlib
import functools
import os

import torch

_ENABLED = os.environ.get("APEX_PROF_RANGES", "0") == "1"


def enable(flag=True):
    global _ENABLED
    _ENABLED = bool(flag)


def enabled():
    return _ENABLED


def _push(name):
    try:
        torch.cuda.nvtx.range_push(name)
        return True
    except Exception:  # no roctx in this build / no GPU
        return False


@contextlib.contextmanager
def range(name):  # noqa: A001 - mirrors nvtx naming
    if not _ENABLED:
        yield
        return
    pushed = _push(name)
    with torch.profiler.record_function(name):
        try:
            yield
        finally:
            if pushed:
                torch.cuda.nvtx.range_pop()


def annotate(name=None):
    """Decorator form of :func:`range`."""

    def deco(fn):
        label = name or fn.__qualname__

        @functools.wraps(fn)
        def wrapper(*a, **k):
            with range(label):
                return fn(*a, **k)

        return wrapper

    return deco
