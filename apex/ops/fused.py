"""Functional fused ops used by the model zoo.

Each op dispatches to the HIP kernel in apex._C for device tensors (when the kernel
exists for that shape) and to the PyTorch reference formulation otherwise; the
reference formulation is what the numerics tests compare against.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import _ext


def attention_qkv_packed(qkv, attn_bias=None, dropout_p=0.0, causal=False, scale=None):
    """qkv: [B, S, 3, h, d] -> context [B, S, h, d]."""
    from ..contrib.multihead_attn import attention as _attn

    return _attn.attention_packed(qkv, attn_bias, dropout_p, causal, scale)


def dropout_add(x, residual, p, training=True):
    """residual + dropout(x)."""
    if p > 0.0 and training:
        return residual + F.dropout(x, p, True)
    return residual + x


def linear_gelu(x, weight, bias):
    """gelu(x @ W^T + b) (erf GELU, as in BERT/GPT-2 exact formulations)."""
    return F.gelu(F.linear(x, weight, bias))


def softmax_cross_entropy(logits, labels, ignore_index=-100, smoothing=0.0, reduction="mean"):
    """Cross entropy with fp32 softmax statistics (apex.contrib.xentropy semantics)."""
    from ..contrib.xentropy import softmax_xentropy

    return softmax_xentropy(logits, labels, smoothing, ignore_index, reduction)
