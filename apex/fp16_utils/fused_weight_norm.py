"""Fused_Weight_Norm (R-14 / K-03): ``w = g * v / ||v||``, norm over every dim but ``dim``.

The reference shipped a stub that raised NotImplementedError
(apex/fp16_utils/fused_weight_norm.py:5-23), which left WeightNorm unusable. Here the
forward/backward run in csrc/norm_misc.hip (``dim == 0``: one norm per output row;
``dim == last``: one norm per column; fp32 accumulation for fp16/bf16 weights). Other
``dim`` values and CPU tensors use the PyTorch reference below.
"""
from __future__ import annotations

import torch

from .. import _ext


def _norm_except_dim(v, dim):
    """Reference ``_norm`` (apex/reparameterization/weight_norm.py:8-18), fp32."""
    if dim is None:
        return v.float().norm()
    d = dim if dim >= 0 else dim + v.dim()
    dims = [x for x in range(v.dim()) if x != d]
    if not dims:
        return v.float().abs()
    shape = [1] * v.dim()
    shape[d] = v.size(d)
    return v.float().pow(2).sum(dims).sqrt().view(shape)


def _mode(v, dim):
    if dim is None or v.dim() < 2:
        return None
    d = dim if dim >= 0 else dim + v.dim()
    if d == 0:
        return True   # row mode
    if d == v.dim() - 1:
        return False  # column mode
    return None


class Fused_Weight_Norm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, g, dim=0):
        mode = _mode(input, dim)
        ctx.dim = dim
        if mode is not None and _ext.use_native(input):
            w, norms = _ext.require().weight_norm_fwd(input, g, mode)
            ctx.save_for_backward(input, g, norms)
            ctx.native = mode
            return w.view_as(input)
        ctx.native = None
        norms = _norm_except_dim(input, dim)
        ctx.save_for_backward(input, g, norms)
        return (input.float() * (g.float() / norms)).to(input.dtype)

    @staticmethod
    def backward(ctx, grad_output):
        input, g, norms = ctx.saved_tensors
        if ctx.native is not None:
            dv, dg = _ext.require().weight_norm_bwd(grad_output, input, g, norms, ctx.native)
            return dv.view_as(input), dg.view_as(g), None
        dim = ctx.dim
        v, go, gf = input.float(), grad_output.float(), g.float()
        if dim is None:
            dims = list(range(v.dim()))
        else:
            d = dim if dim >= 0 else dim + v.dim()
            dims = [x for x in range(v.dim()) if x != d]
        dot = (go * v).sum(dims, keepdim=True) if dims else go * v
        grad_g = dot / norms
        grad_v = (gf / norms) * (go - v * (dot / (norms * norms)))
        return grad_v.to(input.dtype), grad_g.to(g.dtype).view_as(g), None
