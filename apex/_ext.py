"""Loader for the in-tree HIP extension ``apex._C`` (built by tools/build_ext.py).

Policy (MI355X-first, no silent fallbacks on the GPU):
  * on a machine with a ROCm GPU, a missing/broken ``apex._C`` is a hard error the
    first time a fused op is used (``require()``), so a GPU run can never pass on an
    eager-PyTorch stand-in;
  * on a CPU-only machine ops that have a CPU meaning (amp on CPU tensors, O0, the
    plumbing config of BASELINE.json) run their PyTorch reference path, which is also
    the fp32 numerics reference used by the tests.
"""
from __future__ import annotations

import importlib
import os

_C = None
_err: Exception | None = None


def _load():
    global _C, _err
    if _C is not None or _err is not None:
        return _C
    try:
        import torch  # noqa: F401  (torch must load its HIP runtime first)

        so = os.environ.get("APEX_EXT_SO")  # A/B runs: load another build of the same module
        if so:
            import importlib.util as ilu
            import sys

            spec = ilu.spec_from_file_location("apex._C", so)
            _C = ilu.module_from_spec(spec)
            spec.loader.exec_module(_C)
            sys.modules["apex._C"] = _C
        else:
            _C = importlib.import_module("apex._C")
    except Exception as e:  # pragma: no cover - depends on build state
        _err = e
    return _C


def available() -> bool:
    return _load() is not None


def require():
    """Return the extension module or raise loudly."""
    m = _load()
    if m is None:
        raise RuntimeError(
            "apex._C (MI355X HIP kernels) is not built or failed to load: "
            f"{_err!r}. Run `python tools/build_ext.py` (hipcc --offload-arch=gfx950).")
    return m


def use_native(*tensors) -> bool:
    """True when the fused HIP path must be used for these tensors.

    Device tensors always take the native path (and fail loudly when it is
    missing); CPU tensors take the PyTorch reference path.
    ``APEX_FORCE_REFERENCE=1`` forces the reference path (debug only).
    """
    if os.environ.get("APEX_FORCE_REFERENCE", "0") == "1":
        return False
    for t in tensors:
        if t is not None and getattr(t, "is_cuda", False):
            require()
            return True
    return False
