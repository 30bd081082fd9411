"""Autograd wrapper over the MFMA flash-attention kernels (csrc/attention.hip)."""
from __future__ import annotations

import math

import torch

from ... import _ext


def _seed_pair(p, device=None):
    if p <= 0.0:
        return 0, 0
    # from the device generator (apex.utils.rng): reproducible under torch.manual_seed, per-TP-rank
    # inside the RNG tracker's fork, replayed by activation checkpointing; no device sync
    from ...utils.rng import philox_seed_offset

    return philox_seed_offset(device)


def _dbias_buffer(ctx, bias, idx):
    """Zeroed fp32 gradient buffer of the bias's (broadcast) sizes when the bias needs a gradient;
    the backward kernels add dS into it."""
    if bias is None or not ctx.needs_input_grad[idx]:
        return None
    return torch.zeros(bias.shape, dtype=torch.float32, device=bias.device)


def _dbias_out(dbias, bias):
    return None if dbias is None else dbias.to(bias.dtype)


class FlashAttnFunc(torch.autograd.Function):
    """q, k, v: [B, S, H, D] views (D contiguous) -> o [B, Sq, H, D]; ``bias``: optional additive
    score bias (apex.contrib.multihead_attn.attention.prepare_bias layout); when it requires a
    gradient the backward returns dS reduced to its shape."""

    @staticmethod
    def forward(ctx, q, k, v, dropout_p, causal, scale, k_lens, bias=None):
        C = _ext.require()
        seed, offset = _seed_pair(dropout_p, q.device)
        o, lse, dmask = C.flash_attn_fwd(q, k, v, bool(causal), float(scale), float(dropout_p), seed, offset,
                                         k_lens, bias)
        ctx.save_for_backward(q, k, v, o, lse, k_lens, dmask, bias)
        ctx.cfg = (dropout_p, causal, scale, seed, offset)
        return o

    @staticmethod
    def backward(ctx, do):
        C = _ext.require()
        q, k, v, o, lse, k_lens, dmask, bias = ctx.saved_tensors
        p, causal, scale, seed, offset = ctx.cfg
        do = do.contiguous() if do.stride(-1) != 1 else do
        dq = torch.empty_like(q, memory_format=torch.contiguous_format) if not q.is_contiguous() else torch.empty_like(q)
        dk = torch.empty_like(k, memory_format=torch.contiguous_format) if not k.is_contiguous() else torch.empty_like(k)
        dv = torch.empty_like(v, memory_format=torch.contiguous_format) if not v.is_contiguous() else torch.empty_like(v)
        dbias = _dbias_buffer(ctx, bias, 7)
        C.flash_attn_bwd(do, q, k, v, o, lse, dq, dk, dv, bool(causal), float(scale), float(p), seed,
                         offset, k_lens, dmask, None, 0, bias, dbias=dbias)
        return dq, dk, dv, None, None, None, None, _dbias_out(dbias, bias)


class FlashAttnPackedFunc(torch.autograd.Function):
    """qkv: [B, S, 3, H, D] (the fused QKV projection output, consumed in place).
    The gradient is produced directly in the packed [B, S, 3, H, D] layout (no cat)."""

    @staticmethod
    def forward(ctx, qkv, dropout_p, causal, scale, k_lens, bias=None):
        C = _ext.require()
        q, k, v = qkv.unbind(2)
        seed, offset = _seed_pair(dropout_p, qkv.device)
        o, lse, dmask = C.flash_attn_fwd(q, k, v, bool(causal), float(scale), float(dropout_p), seed, offset,
                                         k_lens, bias)
        ctx.save_for_backward(qkv, o, lse, k_lens, dmask, bias)
        ctx.cfg = (dropout_p, causal, scale, seed, offset)
        return o

    @staticmethod
    def backward(ctx, do):
        C = _ext.require()
        qkv, o, lse, k_lens, dmask, bias = ctx.saved_tensors
        p, causal, scale, seed, offset = ctx.cfg
        if do.stride(-1) != 1 or do.stride(1) % 8 or do.stride(0) % 8 or do.stride(2) % 8:
            do = do.contiguous()
        q, k, v = qkv.unbind(2)
        dqkv = torch.empty(qkv.shape, dtype=qkv.dtype, device=qkv.device)
        dq, dk, dv = dqkv.unbind(2)
        dbias = _dbias_buffer(ctx, bias, 5)
        C.flash_attn_bwd(do, q, k, v, o, lse, dq, dk, dv, bool(causal), float(scale), float(p), seed,
                         offset, k_lens, dmask, None, 0, bias, dbias=dbias)
        return dqkv, None, None, None, None, _dbias_out(dbias, bias)


def flash_attention_packed(qkv, dropout_p=0.0, causal=False, scale=None, k_lens=None, bias=None):
    d = qkv.shape[-1]
    scale = 1.0 / math.sqrt(d) if scale is None else scale
    return FlashAttnPackedFunc.apply(qkv, float(dropout_p), bool(causal), float(scale), k_lens, bias)


def flash_attention(q, k, v, dropout_p=0.0, causal=False, scale=None, k_lens=None, bias=None):
    d = q.shape[-1]
    scale = 1.0 / math.sqrt(d) if scale is None else scale
    return FlashAttnFunc.apply(q, k, v, float(dropout_p), bool(causal), float(scale), k_lens, bias)
