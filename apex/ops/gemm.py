"""Dense-layer GEMMs on the hand-written MFMA kernel (csrc/gemm.hip) with fused epilogues.

  linear(x, W, b)              y = x W^T (+ b)                      EPI_NONE / EPI_BIAS
  linear_gelu(x, W, b)         h = x W^T + b, y = gelu(h) -> (y, h)  EPI_BIAS_GELU
  dgrad(dy, W)                 dx = dy W        (via W^T, K-contiguous)
  dgrad_resid(dy, W, r)        dx = dy W + r                         EPI_RESID
  dgrad_dgelu(dy, W, h)        dh = (dy W) * gelu'(h), db = sum(dh)  EPI_DGELU
  linear_gelu_d(x, W, b)       y = gelu(h), g = gelu'(h) -> (y, g)   EPI_BIAS_GELU_D
  dgrad_mul(dy, W, g)          dh = (dy W) * g, db = sum(dh)          EPI_MUL

The kernel takes both operands K-contiguous (A[M,K], B[N,K]); the input-gradient GEMMs use a
transposed copy of W made by a HIP transpose kernel (cheap next to the GEMM: 2 bytes/weight
each way). Weight gradients (contraction over tokens) go through apex.ops.fused._wgrad: the
transposed-read MFMA kernel for the shapes where it wins (BERT-Large's FFN weights), hipBLASLt
split-K otherwise.

Policy (``APEX_GEMM``):
  auto (default)  the MFMA kernel where its fused epilogue removes a separate [M, N] pass
                  (bias+GELU, dGELU+bias-grad, residual add), the library GEMM for plain and
                  bias-only products, where hipBLASLt's assembly main loop is faster than ours.
                  Measured per call on MI355X, BERT-Large layer at M = 32768
                  (tools/gemm_policy_bench.py, profiles/r1_gemm_policy.jsonl):
                    library wins   qkv fwd 164 vs 177 us, attn-out fwd 56 vs 60, FFN2 fwd 180 vs 209,
                                   attn-out dgrad 66 vs 66 (+ transpose)
                    MFMA wins      FFN1 fwd+bias+GELU 299 vs 328 (mm + bias_act), FFN2 dgrad+dGELU
                                   318 vs 402 (mm + bias_act_bwd), QKV dgrad+residual 171 vs 199
                                   (addmm), FFN1 dgrad+residual 221 vs 242
                  Re-measured in round 4 with the balanced main loop at the bench's M = 98304
                  (profiles/r4_gemm_policy_m98304.jsonl): the library still wins the plain
                  products (qkv fwd 476 vs 532 us, attn-out fwd 168 vs 192, FFN2 fwd 551 vs 599);
                  the fused ones are MFMA by 16-24 % (QKV dgrad+residual 482 vs 570, FFN1
                  dgrad+residual 613 vs 717, FFN2 dgrad+dGELU 927 vs 1222, FFN1 fwd+GELU 874 vs 990).
                  What the plain products lose to is the epilogue: the 256-tile rounds store their
                  outputs all at once with the matrix cores idle (19-28 % of the kernel at K = 1024,
                  profiles/r4_gemmlab_ablation_m98304.jsonl).
  mfma            every supported GEMM on the MFMA kernels, including the weight gradients on
                  the transposed-read variant (C.gemm_tt: 266-273 us vs the library's 267-272
                  for the FFN shapes with 4 K-slices; slower for QKV) — A/B and coverage runs
  blas            library GEMM + separate HIP epilogue kernels everywhere
Each function falls back to the library path when the operands do not fit the MFMA kernel
(K % 64, N % 8, dtype, alignment). Numerics follow the unfused composition: the GEMM result is
rounded to the activation dtype before the bias/activation.

FP8: every function takes ``f8`` (an apex.fp8.Fp8State, captured by the calling autograd
Function's forward from ``fp8_state()``); when given and the shapes fit (contraction % 128), the
product runs on the scaled-MFMA fp8 kernel with the same fused epilogue — forward operands e4m3,
backward dy e5m2 x W^T e4m3 — and falls through to the bf16 paths otherwise.
"""
from __future__ import annotations

import os

import torch

from .. import _ext

_MODE = os.environ.get("APEX_GEMM", "auto")
# plain / bias-only products in auto mode: "lib" (hipBLASLt) or "own" (the persistent MFMA kernel)
_PLAIN = os.environ.get("APEX_GEMM_PLAIN", "lib")
# ... except the vocabulary projections measured to win on the MFMA kernel, keyed on the weight's exact
# shape [V, H] (plain forward and input gradient of that weight): BERT-Large's MLM decoder (30522
# padded to 30528 rows): the library's kernels ran 0.93 PF/s there in the BERT step
# (profiles/r5_bert_b768_step_kernels_persist.txt: 985 us forward) against 788 us forward / 648 us dgrad
# on the MFMA kernel (profiles/r5_vocab_gemm_ab.jsonl). GPT-2's LM head measured neutral there, so it
# is not listed, and no width threshold moves unmeasured shapes (a 16384-wide FFN) off the library.
# APEX_GEMM_VOCAB_TABLE = "VxH,..." ("none": empty).
def _parse_shapes(spec):
    out = set()
    for item in spec.split(","):
        item = item.strip()
        if item and item != "none":
            v, h = item.split("x")
            out.add((int(v), int(h)))
    return out


_VOCAB_MEASURED = _parse_shapes(os.environ.get("APEX_GEMM_VOCAB_TABLE", "30528x1024"))


def _vocab_sized(w):
    return tuple(w.shape) in _VOCAB_MEASURED


def _C():
    return _ext.require()


def _2d(x):
    return x.reshape(-1, x.shape[-1])


def mode() -> str:
    return _MODE


def use_mfma(a, w, fused=True, vocab=None) -> bool:
    """MFMA kernel for this call? ``fused``: the call carries an epilogue the library lacks;
    ``vocab``: the (untransposed) weight is a measured vocabulary projection (default: look at w)."""
    vocab = _vocab_sized(w) if vocab is None else vocab
    if _MODE == "blas" or not a.is_cuda or (_MODE == "auto" and not fused and _PLAIN != "own" and not vocab):
        return False
    return _C().gemm_supported(a, w)


def fp8_state():
    """The active apex.fp8 state (None: bf16)."""
    from .. import fp8

    return fp8.active()


def transpose(w):
    """W^T contiguous (HIP transpose kernel for 16-bit dtypes)."""
    if w.is_cuda and w.dtype in (torch.bfloat16, torch.float16) and w.dim() == 2:
        return _C().transpose(w)
    return w.t().contiguous()


def linear(x, w, b=None, f8=None):
    """x [..., K] @ w[N, K]^T (+ b) in x's dtype."""
    a = _2d(x)
    if f8 is not None:
        C = _C()
        r = f8.forward_gemm(a, w, C.EPI_BIAS if b is not None else C.EPI_NONE, b)
        if r is not None:
            return r[0].view(*x.shape[:-1], w.shape[0])
    if use_mfma(a, w, fused=False) and (b is None or b.dtype == x.dtype):
        C = _C()
        y, _ = C.gemm(a, w, C.EPI_BIAS if b is not None else C.EPI_NONE, b)
    else:
        y = torch.addmm(b, a, w.t()) if b is not None else torch.mm(a, w.t())
    return y.view(*x.shape[:-1], w.shape[0])


ACT_GELU, ACT_GELU_TANH = 0, 1  # apex.ops.fused activation codes


def linear_gelu(x, w, b, act=ACT_GELU, f8=None, q8=None):
    """(gelu(h), h) with h = x w^T + b (erf GELU, or tanh GELU for act=1); h kept for backward.
    ``q8``: fp8 side output of gelu(h) on the fp8 path (apex.fp8 producer-side codes)."""
    a = _2d(x)
    C = _C()
    shp = (*x.shape[:-1], w.shape[0])
    r = f8.forward_gemm(a, w, C.EPI_BIAS_GELU_TANH if act == ACT_GELU_TANH else C.EPI_BIAS_GELU, b, q8=q8) \
        if f8 is not None and b is not None else None
    if r is not None:
        return r[0].view(shp), r[1].view(shp)
    if use_mfma(a, w) and b is not None and b.dtype == x.dtype:
        y, h = C.gemm(a, w, C.EPI_BIAS_GELU_TANH if act == ACT_GELU_TANH else C.EPI_BIAS_GELU, b)
    else:
        h = torch.mm(a, w.t())
        y = C.bias_act_fwd(h, b, act)
        h = h + b if b is not None else h  # the pre-activation as the fused path stores it
    shp = (*x.shape[:-1], w.shape[0])
    return y.view(shp), h.view(shp)


def linear_gelu_d(x, w, b, act=ACT_GELU, f8=None, q8=None, codes_only=False):
    """(gelu(h), gelu'(h)) with h = x w^T + b: the forward of an MLP whose backward multiplies by
    the stored derivative (dgrad_mul) instead of re-evaluating erf/exp from h. The derivative
    is taken at the rounded h, as the unfused composition's backward would. ``codes_only`` (fp8,
    with ``q8``): gelu(h) is left unwritten on the fp8 kernel — only its codes are stored."""
    a = _2d(x)
    C = _C()
    shp = (*x.shape[:-1], w.shape[0])
    r = f8.forward_gemm(a, w, C.EPI_BIAS_GELU_TANH_D if act == ACT_GELU_TANH else C.EPI_BIAS_GELU_D, b, q8=q8,
                        codes_only=codes_only) if f8 is not None and b is not None else None
    if r is not None:
        return r[0].view(shp), r[1].view(shp)
    if use_mfma(a, w) and b is not None and b.dtype == x.dtype:
        y, gd = C.gemm(a, w, C.EPI_BIAS_GELU_TANH_D if act == ACT_GELU_TANH else C.EPI_BIAS_GELU_D, b)
    else:
        h = torch.mm(a, w.t())
        y = C.bias_act_fwd(h, b, act)
        gd, _ = C.bias_act_bwd(torch.ones_like(h), h, b, act)  # gelu'(h + b)
    shp = (*x.shape[:-1], w.shape[0])
    return y.view(shp), gd.view(shp)


def dgrad_mul(dy, w, gd, bias_dtype, wT=None, f8=None, bias_grad_out=None, q8=None, codes_only=False):
    """(dh, db): dh = (dy @ w) * gd (gd = the stored activation derivative), db = column sums of dh
    (written into ``bias_grad_out`` on the MFMA path when given). ``codes_only`` (fp8, with ``q8``):
    dh is left unwritten on the fp8 kernel — only its codes (and db) are stored."""
    a = _2d(dy)
    g2 = _2d(gd)
    C = _C()
    r = f8.backward_gemm(a, w, C.EPI_MUL, g2, bias_dtype, q8=q8, codes_only=codes_only) if f8 is not None else None
    if r is not None:
        return r
    if _MODE != "blas" and a.is_cuda and g2.is_contiguous() and g2.dtype == a.dtype:
        wT = transpose(w) if wT is None else wT
        if use_mfma(a, wT):
            dh, db = C.gemm(a, wT, C.EPI_MUL, None, g2, bias_dtype, bias_grad_out)
            return dh, db
    dh = torch.mm(a, w) * g2
    db = C.colsum(dh, bias_dtype) if bias_dtype is not None else None
    return dh, db


def dgrad(dy, w, wT=None, f8=None):
    """dy [..., N] @ w [N, K] -> [..., K]."""
    a = _2d(dy)
    if f8 is not None:
        r = f8.backward_gemm(a, w, _C().EPI_NONE)
        if r is not None:
            return r[0].view(*dy.shape[:-1], w.shape[1])
    vocab = _vocab_sized(w)
    if (_MODE == "mfma" or (_MODE == "auto" and (_PLAIN == "own" or vocab))) and a.is_cuda:
        wT = transpose(w) if wT is None else wT
        if use_mfma(a, wT, fused=False, vocab=vocab):
            C = _C()
            out, _ = C.gemm(a, wT, C.EPI_NONE)
            return out.view(*dy.shape[:-1], w.shape[1])
    return torch.mm(a, w).view(*dy.shape[:-1], w.shape[1])


def dgrad_resid(dy, w, r, wT=None, f8=None):
    """dy @ w + r (the residual-branch gradient accumulated in the epilogue)."""
    a = _2d(dy)
    r2 = _2d(r)
    if f8 is not None:
        res = f8.backward_gemm(a, w, _C().EPI_RESID, r2)
        if res is not None:
            return res[0].view(*dy.shape[:-1], w.shape[1])
    if _MODE != "blas" and a.is_cuda and r2.is_contiguous() and r2.dtype == a.dtype:
        wT = transpose(w) if wT is None else wT
        if use_mfma(a, wT):
            C = _C()
            out, _ = C.gemm(a, wT, C.EPI_RESID, None, r2)
            return out.view(*dy.shape[:-1], w.shape[1])
    return torch.addmm(r2, a, w).view(*dy.shape[:-1], w.shape[1])


def dgrad_dgelu(dy, w, h, bias_dtype, wT=None, act=ACT_GELU, f8=None, bias_grad_out=None, q8=None):
    """(dh, db): dh = (dy @ w) * gelu'(h), db = column sums of dh (in bias_dtype; written into
    ``bias_grad_out`` on the MFMA path when given)."""
    a = _2d(dy)
    h2 = _2d(h)
    C = _C()
    r = f8.backward_gemm(a, w, C.EPI_DGELU_TANH if act == ACT_GELU_TANH else C.EPI_DGELU, h2, bias_dtype, q8=q8) \
        if f8 is not None else None
    if r is not None:
        return r
    if _MODE != "blas" and a.is_cuda and h2.is_contiguous() and h2.dtype == a.dtype:
        wT = transpose(w) if wT is None else wT
        if use_mfma(a, wT):
            epi = C.EPI_DGELU_TANH if act == ACT_GELU_TANH else C.EPI_DGELU
            dh, db = C.gemm(a, wT, epi, None, h2, bias_dtype, bias_grad_out)
            return dh, db
    dg = torch.mm(a, w)
    dh, _ = C.bias_act_bwd(dg, h2, None, act)
    db = C.colsum(dh, bias_dtype) if bias_dtype is not None else None
    return dh, db
