"""FusedScaleMaskSoftmax (apex.transformer.functional) over csrc/softmax.hip.

``FusedScaleMaskSoftmax(input_in_fp16, input_in_bf16, attn_mask_type, scaled_masked_softmax_fusion,
mask_func, softmax_in_fp32, scale)``; ``forward(input[b, np, sq, sk], mask[b, 1, sq, sk])``.
Fused path: fp16/bf16 input, sk % 8 == 0 and sk <= 4096 (one wave64 per row in registers);
otherwise the PyTorch formulation (mask_func + softmax in fp32).
"""
from __future__ import annotations

import torch

from ... import _ext
from ..enums import AttnMaskType


class ScaledUpperTriangMaskedSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inputs, scale):
        y = _ext.require().scaled_masked_softmax_fwd(inputs.contiguous(), None, float(scale), 2, 1)
        ctx.save_for_backward(y)
        ctx.scale = scale
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return _ext.require().scaled_masked_softmax_bwd(dy, y, float(ctx.scale)), None


class ScaledMaskedSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inputs, mask, scale):
        heads = inputs.shape[1]
        m = mask.to(torch.uint8).contiguous() if mask.dtype != torch.uint8 else mask.contiguous()
        y = _ext.require().scaled_masked_softmax_fwd(inputs.contiguous(), m, float(scale), 1, heads)
        ctx.save_for_backward(y)
        ctx.scale = scale
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return _ext.require().scaled_masked_softmax_bwd(dy, y, float(ctx.scale)), None, None


class ScaledSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inputs, scale):
        y = _ext.require().scaled_masked_softmax_fwd(inputs.contiguous(), None, float(scale), 0, 1)
        ctx.save_for_backward(y)
        ctx.scale = scale
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return _ext.require().scaled_masked_softmax_bwd(dy, y, float(ctx.scale)), None


class FusedScaleMaskSoftmax(torch.nn.Module):
    def __init__(self, input_in_fp16, input_in_bf16, attn_mask_type, scaled_masked_softmax_fusion, mask_func,
                 softmax_in_fp32, scale):
        super().__init__()
        self.input_in_fp16 = input_in_fp16
        self.input_in_bf16 = input_in_bf16
        if input_in_fp16 and input_in_bf16:
            raise RuntimeError("both fp16 and bf16 flags cannot be active at the same time.")
        self.input_in_float16 = input_in_fp16 or input_in_bf16
        self.attn_mask_type = attn_mask_type
        self.scaled_masked_softmax_fusion = scaled_masked_softmax_fusion
        self.mask_func = mask_func
        self.softmax_in_fp32 = softmax_in_fp32
        self.scale = scale
        if not (scale is None or softmax_in_fp32):
            raise RuntimeError("softmax should be in fp32 when scaled")

    def forward(self, input, mask):
        assert input.dim() == 4
        if input.is_cuda and self.is_kernel_available(mask, *input.size()):
            return self.forward_fused_softmax(input, mask)
        return self.forward_torch_softmax(input, mask)

    def is_kernel_available(self, mask, b, np, sq, sk):
        if not (self.scaled_masked_softmax_fusion and self.input_in_float16 and input_is_native()):
            return False
        C = _ext.require()
        if not C.scaled_softmax_supported(sk):
            return False
        if self.attn_mask_type == AttnMaskType.causal:
            return sq == sk
        return True

    def forward_fused_softmax(self, input, mask):
        scale = self.scale if self.scale is not None else 1.0
        if self.attn_mask_type == AttnMaskType.causal:
            return ScaledUpperTriangMaskedSoftmax.apply(input, scale)
        if mask is not None:
            return ScaledMaskedSoftmax.apply(input, mask, scale)
        return ScaledSoftmax.apply(input, scale)

    def forward_torch_softmax(self, input, mask):
        if self.input_in_float16 and self.softmax_in_fp32:
            input = input.float()
        if self.scale is not None:
            input = input * self.scale
        if self.attn_mask_type == AttnMaskType.causal and mask is None:
            sq, sk = input.shape[-2:]
            mask = torch.ones(sq, sk, dtype=torch.bool, device=input.device).triu(1)[None, None]
        mask_output = self.mask_func(input, mask) if mask is not None else input
        probs = torch.nn.Softmax(dim=-1)(mask_output)
        if self.input_in_float16 and self.softmax_in_fp32:
            probs = probs.half() if self.input_in_fp16 else probs.bfloat16()
        return probs

    @staticmethod
    def get_batch_per_block(sq, sk, b, np):
        return 4  # one wave64 per row, 4 rows per 256-thread block


_native_flag = [None]


def input_is_native():
    if _native_flag[0] is None:
        _native_flag[0] = _ext.available()
    return _native_flag[0]
