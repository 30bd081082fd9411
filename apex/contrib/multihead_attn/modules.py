"""apex.contrib.multihead_attn modules (NS-05): SelfMultiheadAttn, EncdecMultiheadAttn.

Time-first [seq, batch, embed] I/O as in apex's contrib API. The fast path is:
fused input projection (one GEMM for QKV, or Q + one KV GEMM for enc-dec) -> MFMA flash
attention that reads Q/K/V straight out of the projection output through strides (no
split / transpose copies) -> output projection with the bias gradient folded into a HIP
column-sum; with ``include_norm_add`` the pre-LayerNorm is the HIP FusedLayerNorm and the
residual + dropout epilogue is one fused kernel each way.
Key padding masks ([B, Sk], nonzero = padded) become an additive [B, 1, 1, Sk] bias (any padding
pattern, no host synchronisation), combined with ``attn_mask`` (bool: True = masked; float:
additive when ``mask_additive``, else nonzero = masked) inside the flash kernel.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F
from torch import nn

from ...normalization import FusedLayerNorm
from ...ops import fused as fops
from . import attention as _attn


def _bias_from_attn_mask(attn_mask, dtype, additive=True):
    if attn_mask is None:
        return None
    if attn_mask.dtype == torch.bool or not additive:
        masked = attn_mask if attn_mask.dtype == torch.bool else attn_mask != 0
        return torch.zeros(attn_mask.shape, dtype=dtype, device=attn_mask.device).masked_fill(masked, float("-inf"))
    return attn_mask.to(dtype)


def _combined_bias(attn_mask, key_padding_mask, dtype, additive=True):
    """[Sq, Sk] / [B|1, H|1, Sq, Sk] attn_mask and [B, Sk] key_padding_mask -> one additive bias."""
    bias = _bias_from_attn_mask(attn_mask, dtype, additive)
    if key_padding_mask is not None:
        kp = key_padding_mask if key_padding_mask.dtype == torch.bool else key_padding_mask != 0
        kb = torch.zeros(kp.shape, dtype=dtype, device=kp.device).masked_fill(kp, float("-inf"))[:, None, None, :]
        if bias is None:
            bias = kb
        else:
            while bias.dim() < 4:
                bias = bias.unsqueeze(0)
            bias = bias + kb
    return bias


class SelfMultiheadAttn(nn.Module):
    def __init__(self, embed_dim, num_heads, dropout=0.0, bias=False, include_norm_add=False,
                 impl="fast", separate_qkv_params=False, mask_additive=False):
        super().__init__()
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.dropout = dropout
        self.head_dim = embed_dim // num_heads
        assert self.head_dim * num_heads == embed_dim, "embed_dim must be divisible by num_heads"
        self.bias = bias
        self.include_norm_add = include_norm_add
        self.impl = impl
        self.scaling = self.head_dim ** -0.5
        self.separate_qkv_params = separate_qkv_params
        self.mask_additive = mask_additive
        if separate_qkv_params:
            self.q_weight = nn.Parameter(torch.empty(embed_dim, embed_dim))
            self.k_weight = nn.Parameter(torch.empty(embed_dim, embed_dim))
            self.v_weight = nn.Parameter(torch.empty(embed_dim, embed_dim))
        else:
            self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.out_proj_weight = nn.Parameter(torch.empty(embed_dim, embed_dim))
        if bias:
            if separate_qkv_params:
                self.q_bias = nn.Parameter(torch.empty(embed_dim))
                self.k_bias = nn.Parameter(torch.empty(embed_dim))
                self.v_bias = nn.Parameter(torch.empty(embed_dim))
            else:
                self.in_proj_bias = nn.Parameter(torch.empty(3 * embed_dim))
            self.out_proj_bias = nn.Parameter(torch.empty(embed_dim))
        else:
            self.register_parameter("in_proj_bias", None)
            self.register_parameter("out_proj_bias", None)
        if include_norm_add:
            self.lyr_nrm = FusedLayerNorm(embed_dim)
        self.reset_parameters()

    def reset_parameters(self):
        if self.separate_qkv_params:
            for w in (self.q_weight, self.k_weight, self.v_weight):
                nn.init.xavier_uniform_(w, gain=math.sqrt(2))
        else:
            nn.init.xavier_uniform_(self.in_proj_weight, gain=math.sqrt(2))
        nn.init.xavier_uniform_(self.out_proj_weight)
        if self.bias:
            for n in ("in_proj_bias", "q_bias", "k_bias", "v_bias", "out_proj_bias"):
                if getattr(self, n, None) is not None:
                    nn.init.constant_(getattr(self, n), 0.0)

    def _in_proj(self):
        if self.separate_qkv_params:
            w = torch.cat([self.q_weight, self.k_weight, self.v_weight], 0)
            b = torch.cat([self.q_bias, self.k_bias, self.v_bias], 0) if self.bias else None
            return w, b
        return self.in_proj_weight, self.in_proj_bias

    def forward(self, query, key=None, value=None, key_padding_mask=None, need_weights=False,
                attn_mask=None, is_training=True, causal=False):
        S, B, E = query.shape
        p = self.dropout if (is_training and self.training) else 0.0
        x = self.lyr_nrm(query) if self.include_norm_add else query
        w, b = self._in_proj()
        qkv = fops.fused_dense(x, w, b).view(S, B, 3, self.num_heads, self.head_dim)
        q, k, v = (t.transpose(0, 1) for t in qkv.unbind(2))  # [B, S, H, D] strided views
        bias = _combined_bias(attn_mask, key_padding_mask, q.dtype, self.mask_additive)
        ctx = _attn.attention(q, k, v, bias, p, causal, self.scaling)
        ctx = ctx.transpose(0, 1).reshape(S, B, E)
        if self.include_norm_add:
            return fops.bias_dropout_add(fops.fused_dense(ctx, self.out_proj_weight, None),
                                         self.out_proj_bias, query, p), None
        return fops.fused_dense(ctx, self.out_proj_weight, self.out_proj_bias), None


class EncdecMultiheadAttn(nn.Module):
    def __init__(self, embed_dim, num_heads, dropout=0.0, bias=False, include_norm_add=False, impl="fast"):
        super().__init__()
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.dropout = dropout
        self.head_dim = embed_dim // num_heads
        assert self.head_dim * num_heads == embed_dim, "embed_dim must be divisible by num_heads"
        self.bias = bias
        self.include_norm_add = include_norm_add
        self.impl = impl
        self.scaling = self.head_dim ** -0.5
        self.in_proj_weight_q = nn.Parameter(torch.empty(embed_dim, embed_dim))
        self.in_proj_weight_kv = nn.Parameter(torch.empty(2 * embed_dim, embed_dim))
        self.out_proj_weight = nn.Parameter(torch.empty(embed_dim, embed_dim))
        if bias:
            self.in_proj_bias_q = nn.Parameter(torch.empty(embed_dim))
            self.in_proj_bias_kv = nn.Parameter(torch.empty(2 * embed_dim))
            self.out_proj_bias = nn.Parameter(torch.empty(embed_dim))
        else:
            self.register_parameter("in_proj_bias_q", None)
            self.register_parameter("in_proj_bias_kv", None)
            self.register_parameter("out_proj_bias", None)
        if include_norm_add:
            self.lyr_nrm = FusedLayerNorm(embed_dim)
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.xavier_uniform_(self.in_proj_weight_q)
        nn.init.xavier_uniform_(self.in_proj_weight_kv, gain=math.sqrt(1.5))
        nn.init.xavier_uniform_(self.out_proj_weight)
        if self.bias:
            nn.init.constant_(self.in_proj_bias_q, 0.0)
            nn.init.constant_(self.in_proj_bias_kv, 0.0)
            nn.init.constant_(self.out_proj_bias, 0.0)

    def forward(self, query, key, value=None, key_padding_mask=None, need_weights=False, attn_mask=None,
                is_training=True):
        Sq, B, E = query.shape
        Sk = key.shape[0]
        p = self.dropout if (is_training and self.training) else 0.0
        x = self.lyr_nrm(query) if self.include_norm_add else query
        q = fops.fused_dense(x, self.in_proj_weight_q, self.in_proj_bias_q)
        kv = fops.fused_dense(key, self.in_proj_weight_kv, self.in_proj_bias_kv)
        q = q.view(Sq, B, self.num_heads, self.head_dim).transpose(0, 1)
        k, v = (t.transpose(0, 1) for t in kv.view(Sk, B, 2, self.num_heads, self.head_dim).unbind(2))
        ctx = _attn.attention(q, k, v, _combined_bias(attn_mask, key_padding_mask, q.dtype), p, False,
                              self.scaling)
        ctx = ctx.transpose(0, 1).reshape(Sq, B, E)
        if self.include_norm_add:
            return fops.bias_dropout_add(fops.fused_dense(ctx, self.out_proj_weight, None),
                                         self.out_proj_bias, query, p), None
        return fops.fused_dense(ctx, self.out_proj_weight, self.out_proj_bias), None
