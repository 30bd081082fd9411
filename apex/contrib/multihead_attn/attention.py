"""Attention core used by apex.contrib.multihead_attn and the model zoo (NS-05).

``attention_packed(qkv[B,S,3,h,d], bias, p, causal, scale, k_lens) -> [B,S,h,d]`` and
``attention(q, k, v, ...)`` for separate [B, S, h, d] views.

Every bf16/fp16 device call runs the MFMA flash-attention kernels in apex._C
(csrc/attention_impl.h):

* head dims 32 / 64 / 128 / 256 natively; any other head dim up to 256 (multiple of 8) is
  zero-padded to the next of those (zero columns add nothing to Q K^T, and the padded V columns
  are sliced off the output), with the softmax scale of the ORIGINAL head dim;
* ``attn_bias``: an additive score bias broadcastable to [B, h, Sq, Sk] (attention masks as
  -inf, ALiBi, relative-position biases) is added inside the kernel — no [B, h, Sq, Sk] score
  tensor is materialised; a boolean mask follows scaled_dot_product_attention's convention
  (True = attend) and becomes a 0 / -inf bias. A bias that requires a gradient gets it from the
  backward kernels: dS written into an fp32 tensor of the bias's (broadcast) shape, atomically
  added over the broadcast dims;
* ``k_lens``: per-batch valid key lengths (right padding) skip whole key tiles.

fp32 device inputs (head dims up to 128) run the f32-MFMA flash kernels (csrc/attention_f32.hip:
exact f32 products and accumulation, the same masks / bias / dropout semantics).

Device calls the flash kernels do not take — fp32 head dims > 128, head dims > 256 — run the
query-blocked memory-efficient path (``chunked.chunked_attention``: O(S * block) memory, backward by
recomputation from the saved log-sum-exp, bias gradient = the score gradient), never the O(S^2)
composition. The reference composition (``attention_reference``: matmul -> softmax in fp32 ->
dropout -> matmul) runs on CPU tensors; ``APEX_ATTN_BACKEND=reference`` forces it (A/B, numerics
checks).
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from ... import _ext

_NATIVE_DIMS = (32, 64, 128, 256)


def _padded_dim(d):
    for n in _NATIVE_DIMS:
        if d <= n:
            return n
    return None


def _native_ok(t, bias):
    if os.environ.get("APEX_ATTN_BACKEND", "native") in ("reference", "sdpa", "chunked"):
        return False
    if not t.is_cuda:
        return False
    d = t.shape[-1]
    if d % 8 or _padded_dim(d) is None:
        return False
    if t.dtype == torch.float32:
        # fp32: the f32-MFMA kernels (csrc/attention_f32.hip), head dims up to 128;
        # APEX_ATTN_F32=0 selects the torch compositions (A/B)
        if os.environ.get("APEX_ATTN_F32", "1") == "0" or _padded_dim(d) > 128:
            return False
    elif t.dtype not in (torch.float16, torch.bfloat16):
        return False
    C = _ext._load()
    return C is not None and hasattr(C, "flash_attn_fwd")


def prepare_bias(bias, B, H, Sq, Sk, dtype):
    """An additive bias as a [B|1, H|1, Sq|1, Sk] view in ``dtype`` whose rows the kernel can load
    8 bytes at a time (key-contiguous, row stride a multiple of 4 elements). Broadcast dims keep
    size 1; nothing is expanded to the full score shape."""
    if bias is None:
        return None
    if bias.dtype == torch.bool:
        bias = torch.zeros(bias.shape, dtype=dtype, device=bias.device).masked_fill(~bias, float("-inf"))
    # (no detach: a trainable bias keeps its graph; the flash backward returns dS for this view)
    bias = bias.to(dtype)
    while bias.dim() < 4:
        bias = bias.unsqueeze(0)
    if bias.shape[-1] != Sk:
        bias = bias.expand(*bias.shape[:-1], Sk)
    for dim, full in zip(range(3), (B, H, Sq)):
        if bias.shape[dim] not in (1, full):
            raise ValueError(f"attention bias of shape {tuple(bias.shape)} does not broadcast to "
                             f"[{B}, {H}, {Sq}, {Sk}]")
    ok = bias.stride(-1) == 1 and all(bias.stride(i) % 4 == 0 or bias.shape[i] == 1 for i in range(3)) and \
        bias.data_ptr() % (16 if dtype == torch.float32 else 8) == 0
    if not ok:
        sk4 = (Sk + 3) // 4 * 4
        buf = torch.zeros(*bias.shape[:-1], sk4, dtype=dtype, device=bias.device)
        buf[..., :Sk] = bias
        bias = buf[..., :Sk]
    return bias


def attention_reference(q, k, v, attn_bias=None, dropout_p=0.0, causal=False, scale=None, k_lens=None):
    """q: [B, Sq, h, d], k/v: [B, Sk, h, d] -> [B, Sq, h, d] (fp32 softmax statistics)."""
    B, Sq, H, d = q.shape
    Sk = k.shape[1]
    scale = 1.0 / math.sqrt(d) if scale is None else scale
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) * scale
    if attn_bias is not None:
        bias = attn_bias
        if bias.dtype == torch.bool:
            bias = torch.zeros(bias.shape, device=bias.device).masked_fill(~bias, float("-inf"))
        s = s + bias.float()
    if k_lens is not None:
        km = torch.arange(Sk, device=q.device)[None, :] >= k_lens[:, None].long()
        s = s.masked_fill(km[:, None, None, :], float("-inf"))
    if causal:
        s = s.masked_fill(torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    p = torch.softmax(s, -1).nan_to_num(0.0)  # fully masked rows -> 0, as the kernels do
    if dropout_p > 0:
        p = F.dropout(p, dropout_p, True)
    return torch.einsum("bhqk,bkhd->bqhd", p, v.float()).to(q.dtype)


def _pad_last(t, n):
    return F.pad(t, (0, n - t.shape[-1])) if t.shape[-1] != n else t


def attention_packed(qkv, attn_bias=None, dropout_p=0.0, causal=False, scale=None, k_lens=None):
    B, S, three, h, d = qkv.shape
    scale = 1.0 / math.sqrt(d) if scale is None else scale
    if _native_ok(qkv, attn_bias):
        from . import flash

        bias = prepare_bias(attn_bias, B, h, S, S, qkv.dtype)
        dp = _padded_dim(d)
        if dp == d:
            return flash.flash_attention_packed(qkv, dropout_p, causal, scale, k_lens, bias)
        o = flash.flash_attention_packed(_pad_last(qkv, dp), dropout_p, causal, scale, k_lens, bias)
        return o[..., :d]
    q, k, v = qkv.unbind(2)
    return _fallback(q, k, v, attn_bias, dropout_p, causal, scale, k_lens)


def _short_dense_ok(q, k, attn_bias):
    """Training-length fp32 attention (S <= 1024, fp32 scores of at most 2 GiB, no trainable bias):
    the dense composition — one fused softmax and one fused dropout kernel each way, probabilities
    kept for backward — beats the query-blocked path's recomputation (~3x the elementwise passes
    over [B, h, S, S]): the fp32 BERT-Large step (the bench's speedup denominator, micro-batch 256)
    1741 ms blocked vs 1567 ms dense (BENCH_r02). Longer sequences keep O(S * block) memory."""
    B, Sq, H, _ = q.shape
    Sk = k.shape[1]
    trainable = attn_bias is not None and attn_bias.requires_grad and torch.is_grad_enabled()
    return Sq <= 1024 and Sk <= 1024 and B * H * Sq * Sk * 4 <= (2 << 30) and not trainable


def _fallback(q, k, v, attn_bias, dropout_p, causal, scale, k_lens):
    backend = os.environ.get("APEX_ATTN_BACKEND", "native")
    if q.is_cuda and backend != "reference" and not (backend != "chunked" and _short_dense_ok(q, k, attn_bias)):
        from .chunked import chunked_attention

        return chunked_attention(q, k, v, attn_bias, dropout_p, causal, scale, k_lens)
    return attention_reference(q, k, v, attn_bias, dropout_p, causal, scale, k_lens)


def attention(q, k, v, attn_bias=None, dropout_p=0.0, causal=False, scale=None, k_lens=None):
    """q: [B, Sq, h, d], k/v: [B, Sk, h, d] -> [B, Sq, h, d]."""
    B, Sq, h, d = q.shape
    scale = 1.0 / math.sqrt(d) if scale is None else scale
    if _native_ok(q, attn_bias):
        from . import flash

        bias = prepare_bias(attn_bias, B, h, Sq, k.shape[1], q.dtype)
        dp = _padded_dim(d)
        if dp == d:
            return flash.flash_attention(q, k, v, dropout_p, causal, scale, k_lens, bias)
        o = flash.flash_attention(_pad_last(q, dp), _pad_last(k, dp), _pad_last(v, dp), dropout_p, causal, scale,
                                  k_lens, bias)
        return o[..., :d]
    return _fallback(q, k, v, attn_bias, dropout_p, causal, scale, k_lens)
