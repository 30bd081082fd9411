"""FusedLayerNorm / FusedRMSNorm (NS-03) backed by csrc/layer_norm.hip.

API follows apex.normalization (later apex releases): ``FusedLayerNorm(normalized_shape,
eps=1e-5, elementwise_affine=True)``, ``FusedRMSNorm``, ``MixedFusedLayerNorm`` /
``MixedFusedRMSNorm`` (fp32 params with low-precision activations) and the functional
forms ``fused_layer_norm_affine`` / ``fused_rms_norm_affine`` etc.
"""
from __future__ import annotations

import numbers

import torch
from torch import nn
from torch.nn import init

from .. import _ext


def _cols(normalized_shape) -> int:
    n = 1
    for s in normalized_shape:
        n *= s
    return n


class _FusedNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, normalized_shape, eps, rms):
        C = _ext.require()
        xc = x.contiguous()
        cols = _cols(normalized_shape)
        w = weight.contiguous() if weight is not None else None
        b = bias.contiguous() if bias is not None else None
        y, mean, rstd = C.ln_fwd(xc, cols, w, b, float(eps), bool(rms))
        ctx.save_for_backward(xc, w, b, mean, rstd)
        ctx.cols, ctx.rms = cols, rms
        ctx.params = (weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = _ext.require()
        x, w, b, mean, rstd = ctx.saved_tensors
        from ..ops.fused import _gt

        pw, pb = ctx.params
        # weight / bias gradients straight into their DDP bucket slots when there are any
        dx, dw, db = C.ln_bwd(dy.contiguous(), x, ctx.cols, w, b, mean, rstd, bool(ctx.rms),
                              _gt(pw) if w is not None and ctx.needs_input_grad[1] else None,
                              _gt(pb) if b is not None and ctx.needs_input_grad[2] else None)
        return (dx, dw if w is not None and ctx.needs_input_grad[1] else None,
                db if b is not None and ctx.needs_input_grad[2] else None, None, None, None)


def _ref_rms(x, normalized_shape, weight, eps):
    dims = tuple(range(-len(normalized_shape), 0))
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(dims, keepdim=True) + eps)
    if weight is not None:
        y = y * weight.float()
    return y.to(x.dtype)


def fused_layer_norm_affine(input, weight, bias, normalized_shape, eps=1e-6):
    normalized_shape = _shape(normalized_shape)
    if _ext.use_native(input):
        return _FusedNormFn.apply(input, weight, bias, normalized_shape, eps, False)
    return nn.functional.layer_norm(input, normalized_shape, weight, bias, eps)


def fused_layer_norm(input, normalized_shape, eps=1e-6):
    return fused_layer_norm_affine(input, None, None, normalized_shape, eps)


def fused_rms_norm_affine(input, weight, normalized_shape, eps=1e-6):
    normalized_shape = _shape(normalized_shape)
    if _ext.use_native(input):
        return _FusedNormFn.apply(input, weight, None, normalized_shape, eps, True)
    return _ref_rms(input, normalized_shape, weight, eps)


def fused_rms_norm(input, normalized_shape, eps=1e-6):
    return fused_rms_norm_affine(input, None, normalized_shape, eps)


def mixed_dtype_fused_layer_norm_affine(input, weight, bias, normalized_shape, eps=1e-6):
    return fused_layer_norm_affine(input, weight, bias, normalized_shape, eps)


def mixed_dtype_fused_rms_norm_affine(input, weight, normalized_shape, eps=1e-6):
    return fused_rms_norm_affine(input, weight, normalized_shape, eps)


def _shape(s):
    if isinstance(s, numbers.Integral):
        return (int(s),)
    return tuple(s)


class FusedLayerNorm(nn.Module):
    """Layer normalisation over the trailing ``normalized_shape`` dims (HIP fused)."""

    def __init__(self, normalized_shape, eps=1e-5, elementwise_affine=True, memory_efficient=False):
        super().__init__()
        self.normalized_shape = _shape(normalized_shape)
        self.eps = eps
        self.elementwise_affine = elementwise_affine
        self.memory_efficient = memory_efficient
        if elementwise_affine:
            self.weight = nn.Parameter(torch.empty(*self.normalized_shape))
            self.bias = nn.Parameter(torch.empty(*self.normalized_shape))
        else:
            self.register_parameter("weight", None)
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        if self.elementwise_affine:
            init.ones_(self.weight)
            init.zeros_(self.bias)

    def forward(self, input):
        return fused_layer_norm_affine(input, self.weight, self.bias, self.normalized_shape, self.eps)

    def extra_repr(self):
        return "{normalized_shape}, eps={eps}, elementwise_affine={elementwise_affine}".format(**self.__dict__)


class FusedRMSNorm(nn.Module):
    """RMS normalisation (no mean subtraction, no bias) — HIP fused."""

    def __init__(self, normalized_shape, eps=1e-5, elementwise_affine=True, memory_efficient=False):
        super().__init__()
        self.normalized_shape = _shape(normalized_shape)
        self.eps = eps
        self.elementwise_affine = elementwise_affine
        if elementwise_affine:
            self.weight = nn.Parameter(torch.empty(*self.normalized_shape))
        else:
            self.register_parameter("weight", None)
        self.reset_parameters()

    def reset_parameters(self):
        if self.elementwise_affine:
            init.ones_(self.weight)

    def forward(self, input):
        return fused_rms_norm_affine(input, self.weight, self.normalized_shape, self.eps)

    def extra_repr(self):
        return "{normalized_shape}, eps={eps}, elementwise_affine={elementwise_affine}".format(**self.__dict__)


class MixedFusedLayerNorm(FusedLayerNorm):
    """fp32 affine params with bf16/fp16 activations (output keeps the input dtype)."""

    def __init__(self, normalized_shape, eps=1e-5, **kwargs):
        kwargs.pop("elementwise_affine", None)
        super().__init__(normalized_shape, eps, elementwise_affine=True, **kwargs)

    def _apply(self, fn, recurse=True):
        # keep the affine params fp32 under model.half()/bfloat16()
        w, b = self.weight, self.bias
        out = super()._apply(fn)
        if self.weight.dtype != torch.float32:
            self.weight.data = self.weight.data.float()
            self.bias.data = self.bias.data.float()
        return out


class MixedFusedRMSNorm(FusedRMSNorm):
    def __init__(self, normalized_shape, eps=1e-5, **kwargs):
        kwargs.pop("elementwise_affine", None)
        super().__init__(normalized_shape, eps, elementwise_affine=True, **kwargs)

    def _apply(self, fn, recurse=True):
        out = super()._apply(fn)
        if self.weight.dtype != torch.float32:
            self.weight.data = self.weight.data.float()
        return out
