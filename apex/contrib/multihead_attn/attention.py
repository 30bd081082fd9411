"""Attention core used by apex.contrib.multihead_attn and the model zoo (NS-05).

``attention_packed(qkv[B,S,3,h,d], bias, p, causal, scale) -> [B,S,h,d]``.
Dispatch: the MFMA flash-attention kernels in apex._C (csrc/attention.hip) when
built for the shape; otherwise PyTorch's scaled_dot_product_attention.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ... import _ext


def _native_ok(qkv, bias, p):
    C = _ext._load()
    return C is not None and hasattr(C, "flash_attn_fwd") and qkv.is_cuda and bias is None and \
        qkv.dtype in (torch.float16, torch.bfloat16) and qkv.shape[-1] in (64, 128)


def attention_packed(qkv, attn_bias=None, dropout_p=0.0, causal=False, scale=None):
    B, S, three, h, d = qkv.shape
    if _native_ok(qkv, attn_bias, dropout_p):
        from . import flash

        return flash.flash_attention_packed(qkv, dropout_p, causal, scale)
    q, k, v = qkv.unbind(2)
    q, k, v = (t.transpose(1, 2) for t in (q, k, v))
    mask = None
    if attn_bias is not None:
        mask = attn_bias.to(q.dtype)
    o = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, dropout_p=dropout_p,
                                       is_causal=causal and mask is None, scale=scale)
    return o.transpose(1, 2)


def attention(q, k, v, attn_bias=None, dropout_p=0.0, causal=False, scale=None):
    """q,k,v: [B, S, h, d] -> [B, S, h, d]."""
    if q.shape == k.shape == v.shape and attn_bias is None:
        qkv = torch.stack([q, k, v], dim=2)
        return attention_packed(qkv, attn_bias, dropout_p, causal, scale)
    qt, kt, vt = (t.transpose(1, 2) for t in (q, k, v))
    o = F.scaled_dot_product_attention(qt, kt, vt, attn_mask=attn_bias, dropout_p=dropout_p,
                                       is_causal=causal and attn_bias is None, scale=scale)
    return o.transpose(1, 2)
