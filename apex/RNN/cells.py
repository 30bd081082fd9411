"""RNN cell functions for apex.RNN (R-23, R-27, K-06).

Every cell is "two GEMMs + one fused pointwise kernel": the gate pre-activations come
from ``x W_ih^T`` and ``h W_hh^T`` (library GEMMs), and everything after them — bias adds,
sigmoid/tanh, the cell update, and in backward the gate gradients — is ONE HIP kernel
(csrc/norm_misc.hip lstm_cell_* / gru_cell_*). Bias gradients are column sums of the gate
gradients (HIP colsum). Reference: the THCUNN ``LSTMFused``/``GRUFused`` calls in
apex/RNN/cells.py:60-66 and torch's fused RNN cells used by apex/RNN/models.py:3.
CPU tensors use the plain PyTorch formulation (also the numerics reference).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import _ext


class _LSTMPointwise(torch.autograd.Function):
    @staticmethod
    def forward(ctx, igates, hgates, cx, b_ih, b_hh):
        C = _ext.require()
        hy, cy, ws = C.lstm_cell_fwd(igates, hgates, b_ih, b_hh, cx)
        ctx.save_for_backward(cx, ws)
        ctx.has_h = hgates is not None
        ctx.bias = (b_ih is not None, b_hh is not None)
        ctx.bdt = b_ih.dtype if b_ih is not None else (b_hh.dtype if b_hh is not None else None)
        return hy, cy

    @staticmethod
    def backward(ctx, dhy, dcy):
        C = _ext.require()
        cx, ws = ctx.saved_tensors
        dg, dcx = C.lstm_cell_bwd(dhy, dcy, cx, ws)
        db = C.colsum(dg, ctx.bdt) if any(ctx.bias) else None
        return (dg, dg if ctx.has_h else None, dcx, db if ctx.bias[0] else None,
                db if ctx.bias[1] else None)


class _GRUPointwise(torch.autograd.Function):
    @staticmethod
    def forward(ctx, igates, hgates, hx, b_ih, b_hh):
        C = _ext.require()
        hy, ws = C.gru_cell_fwd(igates, hgates, b_ih, b_hh, hx)
        ctx.save_for_backward(hx, ws)
        ctx.bias = (b_ih is not None, b_hh is not None)
        ctx.bdt = b_ih.dtype if b_ih is not None else (b_hh.dtype if b_hh is not None else None)
        return hy

    @staticmethod
    def backward(ctx, dhy):
        C = _ext.require()
        hx, ws = ctx.saved_tensors
        dig, dhg, dhx = C.gru_cell_bwd(dhy, hx, ws)
        dbi = C.colsum(dig, ctx.bdt) if ctx.bias[0] else None
        dbh = C.colsum(dhg, ctx.bdt) if ctx.bias[1] else None
        return dig, dhg, dhx, dbi, dbh


def _native(x):
    return _ext.use_native(x)


def lstm_pointwise(igates, hgates, cx, b_ih=None, b_hh=None):
    if _native(igates):
        return _LSTMPointwise.apply(igates, hgates, cx, b_ih, b_hh)
    gates = igates + (hgates if hgates is not None else 0)
    if b_ih is not None:
        gates = gates + b_ih
    if b_hh is not None:
        gates = gates + b_hh
    i, f, g, o = gates.chunk(4, 1)
    i, f, g, o = torch.sigmoid(i), torch.sigmoid(f), torch.tanh(g), torch.sigmoid(o)
    cy = f * cx + i * g
    return o * torch.tanh(cy), cy


def gru_pointwise(igates, hgates, hx, b_ih=None, b_hh=None):
    if _native(igates):
        return _GRUPointwise.apply(igates, hgates, hx, b_ih, b_hh)
    gi = igates + (b_ih if b_ih is not None else 0)
    gh = hgates + (b_hh if b_hh is not None else 0)
    ir, iz, inn = gi.chunk(3, 1)
    hr, hz, hn = gh.chunk(3, 1)
    r = torch.sigmoid(ir + hr)
    z = torch.sigmoid(iz + hz)
    n = torch.tanh(inn + r * hn)
    return (1 - z) * n + z * hx


# ---- cell functions with the (input, hidden, w_ih, w_hh, b_ih, b_hh) signature ----------
def LSTMCell(input, hidden, w_ih, w_hh, b_ih=None, b_hh=None):
    hx, cx = hidden
    return lstm_pointwise(F.linear(input, w_ih), F.linear(hx, w_hh), cx, b_ih, b_hh)


def GRUCell(input, hidden, w_ih, w_hh, b_ih=None, b_hh=None):
    return gru_pointwise(F.linear(input, w_ih), F.linear(hidden, w_hh), hidden, b_ih, b_hh)


def RNNReLUCell(input, hidden, w_ih, w_hh, b_ih=None, b_hh=None):
    return F.relu(F.linear(input, w_ih, b_ih) + F.linear(hidden, w_hh, b_hh))


def RNNTanhCell(input, hidden, w_ih, w_hh, b_ih=None, b_hh=None):
    return torch.tanh(F.linear(input, w_ih, b_ih) + F.linear(hidden, w_hh, b_hh))


def mLSTMCell(input, hidden, w_ih, w_hh, w_mih, w_mhh, b_ih=None, b_hh=None):
    """Multiplicative LSTM (reference apex/RNN/cells.py:55-83):
    m = (x W_mih^T) * (h W_mhh^T); gates = x W_ih^T + m W_hh^T (+ biases)."""
    hx, cx = hidden
    m = F.linear(input, w_mih) * F.linear(hx, w_mhh)
    return lstm_pointwise(F.linear(input, w_ih), F.linear(m, w_hh), cx, b_ih, b_hh)
