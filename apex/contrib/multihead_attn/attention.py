"""Attention core used by apex.contrib.multihead_attn and the model zoo (NS-05).

``attention_packed(qkv[B,S,3,h,d], bias, p, causal, scale, k_lens) -> [B,S,h,d]``.
Dispatch: the MFMA flash-attention kernels in apex._C (csrc/attention.hip) for
bf16/fp16 device tensors with head dim 64/128 (key padding expressed as per-batch
``k_lens``); an arbitrary additive ``attn_bias`` or other shapes use PyTorch's
scaled_dot_product_attention. ``APEX_ATTN_BACKEND=sdpa`` forces the latter (A/B).
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from ... import _ext


def _native_ok(t, bias):
    if os.environ.get("APEX_ATTN_BACKEND", "native") == "sdpa":
        return False
    C = _ext._load()
    return C is not None and hasattr(C, "flash_attn_fwd") and t.is_cuda and bias is None and \
        t.dtype in (torch.float16, torch.bfloat16) and t.shape[-1] in (64, 128)


def _lens_to_bias(k_lens, Sk, dtype, device):
    km = torch.arange(Sk, device=device)[None, :] >= k_lens[:, None].long()
    return torch.zeros(km.shape, dtype=dtype, device=device).masked_fill(km, float("-inf"))[:, None, None, :]


def attention_packed(qkv, attn_bias=None, dropout_p=0.0, causal=False, scale=None, k_lens=None):
    B, S, three, h, d = qkv.shape
    if _native_ok(qkv, attn_bias):
        from . import flash

        return flash.flash_attention_packed(qkv, dropout_p, causal, scale, k_lens)
    q, k, v = qkv.unbind(2)
    return _sdpa(q, k, v, attn_bias, dropout_p, causal, scale, k_lens)


def _sdpa(q, k, v, attn_bias, dropout_p, causal, scale, k_lens):
    qt, kt, vt = (t.transpose(1, 2) for t in (q, k, v))
    mask = attn_bias.to(qt.dtype) if attn_bias is not None else None
    if k_lens is not None:
        kb = _lens_to_bias(k_lens, kt.shape[2], qt.dtype, qt.device)
        mask = kb if mask is None else mask + kb
    if causal and mask is not None:
        Sq, Sk = qt.shape[2], kt.shape[2]
        cm = torch.ones(Sq, Sk, dtype=torch.bool, device=qt.device).triu(1)
        mask = mask.masked_fill(cm, float("-inf"))
        causal = False
    o = F.scaled_dot_product_attention(qt, kt, vt, attn_mask=mask, dropout_p=dropout_p,
                                       is_causal=causal, scale=scale)
    return o.transpose(1, 2)


def attention(q, k, v, attn_bias=None, dropout_p=0.0, causal=False, scale=None, k_lens=None):
    """q: [B, Sq, h, d], k/v: [B, Sk, h, d] -> [B, Sq, h, d]."""
    if _native_ok(q, attn_bias):
        from . import flash

        return flash.flash_attention(q, k, v, dropout_p, causal, scale, k_lens)
    return _sdpa(q, k, v, attn_bias, dropout_p, causal, scale, k_lens)
