"""Fused_Weight_Norm (R-14 / K-03): ``w = g * v / ||v||`` over all dims except ``dim``.

The reference shipped a stub that raised NotImplementedError
(apex/fp16_utils/fused_weight_norm.py:5-23), which left WeightNorm unusable. This is a
working autograd function backed by the HIP kernels in csrc/weight_norm.hip.
"""
from __future__ import annotations

import torch

from .. import _ext


def _norm_except_dim(v, dim):
    if dim is None or dim == -1 and v.dim() == 0:
        return v.float().norm()
    if dim < 0:
        dim += v.dim()
    dims = [d for d in range(v.dim()) if d != dim]
    shape = [1] * v.dim()
    shape[dim] = v.size(dim)
    return v.float().pow(2).sum(dims).sqrt().view(shape)


class Fused_Weight_Norm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, g, dim=0):
        if _ext.use_native(input) and hasattr(_ext.require(), "weight_norm_fwd"):
            C = _ext.require()
            w, norms = C.weight_norm_fwd(input.contiguous(), g.contiguous(), int(dim))
            ctx.save_for_backward(input, g, norms)
            ctx.dim = dim
            ctx.native = True
            return w
        norms = _norm_except_dim(input, dim)
        w = (input.float() * (g.float() / norms)).to(input.dtype)
        ctx.save_for_backward(input, g, norms)
        ctx.dim = dim
        ctx.native = False
        return w

    @staticmethod
    def backward(ctx, grad_output):
        input, g, norms = ctx.saved_tensors
        if ctx.native:
            C = _ext.require()
            gi, gg = C.weight_norm_bwd(grad_output.contiguous(), input.contiguous(), g.contiguous(),
                                       norms, int(ctx.dim))
            return gi, gg, None
        dim = ctx.dim
        v = input.float()
        go = grad_output.float()
        if dim is None:
            dims = list(range(v.dim()))
        else:
            d = dim if dim >= 0 else dim + v.dim()
            dims = [x for x in range(v.dim()) if x != d]
        gf = g.float()
        dot = (go * v).sum(dims, keepdim=True) if dims else go * v
        grad_g = dot / norms
        grad_v = (gf / norms) * (go - v * (dot / (norms * norms)))
        return grad_v.to(input.dtype), grad_g.to(g.dtype).view_as(g), None
