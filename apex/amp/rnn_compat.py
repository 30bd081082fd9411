"""RNN support for the amp engine (R-07).

Modern ``torch.nn.RNN/LSTM/GRU`` and the ``*Cell`` modules call into
``torch.nn.modules.rnn._VF`` (``_VF.lstm``, ``_VF.lstm_cell``, ...). ``_VF`` is a
C-extension module whose attributes cannot be wrapped per call site, so amp swaps
in a mutable shim object that forwards to the real ``_VF`` (reference:
apex/amp/rnn_compat.py:14-17) and wraps the shim's entries; ``restore`` undoes it.
"""
from __future__ import annotations

import torch

from . import utils, wrap
from .policy import RNN_NAMES

_ORIG_VF = None


class VariableFunctionsShim:
    """Attribute proxy for torch._VF with writable RNN / RNN-cell entries."""

    def __init__(self, vf):
        self.__dict__["_vf"] = vf
        for name in RNN_NAMES:
            setattr(self, name, getattr(vf, name))
            setattr(self, name + "_cell", getattr(vf, name + "_cell"))

    def __getattr__(self, name):
        return getattr(self.__dict__["_vf"], name)


def has_old_rnns():
    return False


def install_shim():
    global _ORIG_VF
    mod = torch.nn.modules.rnn
    if not isinstance(mod._VF, VariableFunctionsShim):
        _ORIG_VF = mod._VF
        mod._VF = VariableFunctionsShim(mod._VF)
    return mod._VF


def restore():
    global _ORIG_VF
    if _ORIG_VF is not None:
        torch.nn.modules.rnn._VF = _ORIG_VF
        _ORIG_VF = None


def whitelist_rnn_cells(handle, verbose):
    shim = install_shim()
    for name in RNN_NAMES:
        wrap.cached_cast(shim, name + "_cell", utils.maybe_half, handle, try_caching=True,
                         verbose=verbose)


def whitelist_rnns(handle, verbose):
    shim = install_shim()
    for name in RNN_NAMES:
        wrap.rnn_cast(shim, name, handle, verbose)
    # torch>=2 RNNBase.check_input rejects input/weight dtype mismatch unless torch's own
    # autocast is on; under amp the dtype is reconciled by the _VF wrapper instead.
    base = torch.nn.modules.rnn.RNNBase
    orig_check = base.check_input

    def check_input(self, input, batch_sizes):
        if handle.is_active() and input.is_floating_point():
            expected_dim = 2 if batch_sizes is not None else 3
            if input.dim() != expected_dim:
                raise RuntimeError("input must have {} dimensions, got {}".format(expected_dim, input.dim()))
            if self.input_size != input.size(-1):
                raise RuntimeError("input.size(-1) must be equal to input_size. Expected {}, got {}"
                                   .format(self.input_size, input.size(-1)))
            return
        return orig_check(self, input, batch_sizes)

    utils.set_func_save(handle, base, "check_input", check_input)
