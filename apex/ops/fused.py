"""Functional fused ops used by the model zoo (transformer building blocks).

Each op is an autograd Function over the HIP kernels in apex._C for device tensors, and
the PyTorch reference formulation on CPU (also the numerics reference for the tests):

  fused_dense(x, W, b)                      y = x W^T + b            (bias grad: HIP colsum)
  dense_gelu(x, W, b)                       y = gelu(x W^T + b)      (bias+GELU fwd/bwd fused,
                                                                     bias grad folded in)
  bert_embeddings(ids, types, Ww, Wp, Wt, gamma, beta, p, eps)
                                            y = dropout(LN(Ww[ids] + Wp[pos] + Wt[types]))
  dense_bias_dropout_add_ln(x, W, b, res, gamma, beta, p, eps)
                                            y = LN(res + dropout(x W^T + b))  (one fused
                                                                     kernel each way)
  bias_dropout_add(x, b, res, p)            y = res + dropout(x + b)
  attention_qkv_packed / softmax_cross_entropy

Forward and input-gradient GEMMs run on the hand-written MFMA kernel (apex.ops.gemm, with
bias / bias+GELU in its epilogue where it applies); weight gradients are hipBLASLt with split-K.
Dropout masks are regenerated from a Philox key derived from the device's torch generator
(apex.utils.rng), so results are reproducible under ``torch.manual_seed``, differ across
tensor-parallel ranks inside ``get_cuda_rng_tracker().fork()``, and no mask tensor is stored.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .. import _ext

ACT_GELU, ACT_GELU_TANH, ACT_RELU, ACT_NONE = 0, 1, 2, 3


def _seed(device=None):
    """(Philox key, counter base) for one dropout launch: from the device's torch generator
    (apex.utils.rng), so masks follow torch.manual_seed, the TP RNG tracker's fork and
    activation-checkpoint recomputation."""
    from ..utils.rng import philox_seed_offset

    return philox_seed_offset(device)


def _native(*ts):
    return _ext.use_native(*ts)


def _2d(x):
    return x.reshape(-1, x.shape[-1])


_WGRAD_SPLITK = os.environ.get("APEX_WGRAD_SPLITK", "auto")


def _wgrad_splits(M, N, K):
    """K-slices for dW[N,K] = dY[M,N]^T X[M,K] (M = tokens, the contraction).

    A 1024x1024 weight gradient is only 16 output tiles of 256x256 — a sixteenth of the 256
    CUs — however long its M=32k contraction is, so the library GEMM runs at ~0.5 PF/s.
    Slicing M into S batched GEMMs fills the chip (S*tiles ~ 128-256 workgroups); the fp32
    slabs are combined by one HIP reduction that writes the grad dtype. Measured on MI355X
    (tools/gemm_bench.py, BERT-Large shapes, M = 32768): 1024x1024 199 -> 79 us (S=8),
    3072x1024 288 -> 199 us (S=4), 4096x1024 316 -> 262 us (S=4). At M = 98304
    (profiles/r2_wgrad_split_sweep.jsonl, every S dividing M): 1024x1024 best at S=16 (194 us vs
    215 at 8, 499 unsplit), 3072x1024 and the FFN shapes at S=4 — i.e. S*tiles ~ 256 workgroups.
    """
    if _WGRAD_SPLITK == "0":
        return 1
    if _WGRAD_SPLITK not in ("auto", ""):
        s = int(_WGRAD_SPLITK)
        return s if M % s == 0 else 1
    if M < 8192:
        return 1
    tiles = ((N + 255) // 256) * ((K + 255) // 256)
    s = 1
    while s < 16 and 2 * s * tiles <= 256 and M % (2 * s) == 0 and M // (2 * s) >= 1024:
        s *= 2
    return s


_WGRAD_TT = os.environ.get("APEX_WGRAD_TT", "auto")
_WGRAD_TT_VOCAB = os.environ.get("APEX_WGRAD_TT_VOCAB", "1") != "0"


def _wgrad_tt_splits(M, N, K):
    """K-slices for the weight gradient on the transposed-read MFMA kernel (csrc/gemm.hip gemm_tt,
    fp32 slabs + the same splitk_reduce), or 0 to keep the library split-K.
    ``APEX_WGRAD_TT``: auto, 0 (library only), or a slice count. auto: the 256x256-tile counts of
    BERT-Large's FFN weights (64 tiles: 4 slices = one wave of 256 workgroups), where the kernel
    beats hipBLASLt since the balanced main loop (tools/wgrad_tt_bench.py, M = 98304,
    profiles/r4_wgrad_tt_vs_lib.jsonl); the QKV (48 tiles) and output-projection (16) shapes stay on
    the library, which is as fast or faster there. Auto is limited to the measured tile range
    (64 <= tiles < 128); larger weights (hundreds of tiles, e.g. Megatron / GPT MLPs) stay on the
    library until measured."""
    if _WGRAD_TT == "0" or N % 8 or K % 8:
        return 0
    if _WGRAD_TT not in ("auto", ""):
        s = int(_WGRAD_TT)
        return s if M % 64 == 0 and M // 64 >= s else 0
    if _WGRAD_TT_VOCAB and max(N, K) >= 16384 and M % 64 == 0:
        # vocabulary-sized weights (an MLM decoder / LM head tied to the embedding): hundreds of
        # output tiles, one slice (profiles/r5_vocab_wgrad_tt_ab.jsonl: the MLM decoder wgrad 964 -> 795 us)
        return 1
    hit = _WGRAD_TT_MEASURED.get((N, K))
    if hit is not None:
        m_min, s = hit
        return s if M >= m_min and M % 64 == 0 and M // 64 >= s else 0
    if N % 256 or K % 256:
        return 0  # partial tiles run on the kernel (forced counts above); auto keeps measured shapes only
    tiles = (N // 256) * (K // 256)
    if M < 16384 or tiles < 64 or tiles >= 128 or M % 256:
        return 0
    return max(1, 256 // tiles)


# (N, K) -> (min tokens, slices): weight-gradient shapes routed to the transposed-read kernel by
# measurement. Empty: in isolation (tools/wgrad_tt_bench.py, profiles/r5_wgrad_tt_gpt2_megatron.jsonl)
# the kernel beat the library on GPT-2 1.5B's attention-out / FFN shapes (123 vs 142, 379 vs 458, 378 vs
# 490 us at 16384 tokens, partial 256-tiles) and Megatron H2560's (122 vs 136, 437 vs 512 us), but the
# GPT-2 model step with those shapes routed was 1.3 % SLOWER (84.2k vs 85.3k tokens/s, same box,
# profiles/r5_gpt2_wgrad_tt_ab.jsonl; a likely cause, unverified: the isolated loop re-reads the same
# ~260 MB of operands, mostly served from the 256 MB Infinity Cache) — so the library keeps them (forced APEX_WGRAD_TT=<slices>
# still runs any multiple-of-8 shape on the kernel).
# Round 5, after the split-major XCD remap and with the library on its TunableOp selections (the
# isolated tool's 'lib' rows were untuned before: profiles/r5_wgrad_tt_vs_tuned_lib.jsonl): the
# attention-out weight gradients win on the kernel — BERT-Large 1024x1024 at 16 slices 198 vs 226 us,
# GPT-2 1.5B 1600x1600 at 4 slices 117 vs 137 us — and GPT-2's FFN shapes lose (372 / 365 vs 335 / 325).
# APEX_WGRAD_TT_TABLE replaces the table for A/B runs: "NxK:min_tokens:slices,..." ("none": empty).
_WGRAD_TT_MEASURED = {(1024, 1024): (65536, 16), (1600, 1600): (16384, 4)}


def _parse_tt_table(spec):
    table = {}
    for item in spec.split(","):
        item = item.strip()
        if not item or item == "none":
            continue
        try:
            nk, m_min, s = item.split(":")
            n, k = nk.split("x")
            table[(int(n), int(k))] = (int(m_min), int(s))
        except ValueError as e:
            raise ValueError(f"APEX_WGRAD_TT_TABLE entry {item!r}: expected NxK:min_tokens:slices") from e
    return table


if os.environ.get("APEX_WGRAD_TT_TABLE") is not None:
    _WGRAD_TT_MEASURED = _parse_tt_table(os.environ["APEX_WGRAD_TT_TABLE"])


def _gt(p):
    """The parameter's DDP bucket slot to write its gradient into, or None
    (apex.parallel.distributed.grad_target)."""
    from ..parallel.distributed import grad_target

    return grad_target(p) if p is not None else None


_MAIN_GRAD_GEMM = os.environ.get("APEX_MAIN_GRAD_GEMM", "auto")


def _main_grad_tt(M, N, K):
    """fp32 main_grad accumulation on the MFMA kernel (gemm_tt_acc) for this dW[N, K] shape?
    ``APEX_MAIN_GRAD_GEMM``: auto, tt (always when supported), lib (hipBLASLt / split-K slabs only).
    auto: when the 256x256 output tiles fill the 256 CUs' rounds to >= 75 % (one tile per CU and
    round, unsplit). Measured at Megatron H2560, 8192 tokens (profiles/r3_main_grad_ab.jsonl):
    10240x2560 and 2560x10240 (400 tiles, 78 %) 455 vs 531-538 us for hipBLASLt's fp32-output
    addmm; 7680x2560 (300 tiles, 59 %) 455 vs 355 and 2560x2560 (100 tiles) 211 vs 127 — there the
    library keeps them."""
    if _MAIN_GRAD_GEMM == "lib":
        return False
    if _MAIN_GRAD_GEMM == "tt":
        return True
    tiles = (N // 256) * (K // 256)
    rounds = -(-tiles // 256)
    return tiles >= 192 and tiles >= 0.75 * rounds * 256


def accumulate_main_grad(mg, dy2, x2):
    """mg (fp32) += dy2^T @ x2 with fp32 accumulation and no 16-bit rounding: the split-K batched
    GEMM's fp32 slabs (one slab when the shape does not split) summed INTO mg by one HIP pass
    (splitk_reduce accumulate) — the micro-batch gradient accumulation of DDP's fp32_main_grad
    mode, with no separate add kernel and no bf16 dW tensor."""
    M, N = dy2.shape
    K = x2.shape[1]
    if not (dy2.is_cuda and _native(dy2) and dy2.dtype in (torch.bfloat16, torch.float16)
            and dy2.is_contiguous() and x2.is_contiguous() and mg.is_contiguous()):
        mg.add_(dy2.t().float().mm(x2.float()))
        return mg
    if (_main_grad_tt(M, N, K) and mg.dtype == torch.float32 and mg.dim() == 2 and tuple(mg.shape) == (N, K)
            and mg.data_ptr() % 16 == 0 and _ext.require().gemm_tt_supported(dy2, x2, 1)):
        # (gemm_tt_acc's 16-byte read-modify-write epilogue needs main_grad 16-byte aligned and
        # [N, K]: an unaligned user buffer or APEX_DDP_ALIGN=0 slot takes the addmm / split-K path)
        # the transposed-read MFMA kernel with the fp32 read-modify-write epilogue: dW is added
        # into main_grad in the GEMM's own epilogue (csrc/gemm.hip EPI_F32_ACC)
        _ext.require().gemm_tt_acc(dy2, x2, mg)
        return mg
    s = _wgrad_splits(M, N, K)
    if s == 1:
        # enough output tiles to fill the chip: hipBLASLt accumulates straight into main_grad
        # (fp32 C = D, beta = 1) — no slab round trip (tools/main_grad_ab.py, Megatron H2560
        # shapes: 358 vs 441 us at 7680x2560, 529 vs 562 us at 2560x10240; same fp32 error)
        torch.addmm(mg, dy2.t(), x2, out_dtype=torch.float32, out=mg)
        return mg
    slabs = torch.bmm(dy2.view(s, M // s, N).transpose(1, 2), x2.view(s, M // s, K), out_dtype=torch.float32)
    _ext.require().splitk_reduce(slabs, torch.float32, mg, accumulate=True)
    return mg


def main_grad_placeholder(param):
    """The gradient a fused producer hands autograd after accumulating into ``param.main_grad``:
    a storage-less ZeroTensor, so the parameter's AccumulateGrad (and the DDP readiness hook
    behind it) still fires without a fill kernel or a parameter-sized allocation. When the
    parameter has other uses (a tied embedding: the lookup's dense gradient), autograd sums them
    with it and the hook sees an ordinary tensor, which it adds into main_grad — only a bare
    placeholder is dropped (apex.parallel.DistributedDataParallel._grad_hook)."""
    param.grad_added_to_main_grad = True
    return torch._efficientzerotensor(param.shape, dtype=param.dtype, device=param.device)


def _wgrad(dy2, x2, out=None, param=None, f8=None):
    """Weight gradient dy2^T @ x2 in dy2's dtype (split-K batched GEMM when it pays), written into
    ``out`` when given (a gradient-bucket slot), or into ``param``'s bucket slot
    (apex.parallel.grad_target). When ``param`` carries an fp32 ``main_grad`` (DDP
    fp32_main_grad mode) the gradient is accumulated there instead and a placeholder is returned
    for autograd (main_grad_placeholder: the DDP hook drops it). ``f8`` = (Fp8State, dy2 codes,
    x2 codes) (apex.fp8 ``operand_codes``): the product runs on those fp8 codes instead."""
    if param is not None:
        mg = getattr(param, "main_grad", None)
        if mg is not None:
            accumulate_main_grad(mg, dy2, x2)
            return main_grad_placeholder(param)
        if out is None:
            out = _gt(param)
    if f8 is not None and f8[0] is not None and (out is None or out.is_contiguous()):
        r = f8[0].wgrad(f8[1], f8[2], dy2.dtype, out=out)
        if r is not None:
            return r
    M, N = dy2.shape
    K = x2.shape[1]
    s = _wgrad_splits(M, N, K) if dy2.dtype in (torch.bfloat16, torch.float16) else 1
    from . import gemm as G

    if dy2.is_cuda and dy2.dtype in (torch.bfloat16, torch.float16):
        C = _ext.require()
        st = _wgrad_tt_splits(M, N, K)
        if G.mode() == "mfma" and not st:
            st = max(s, 4 if M >= 16384 else 1)
        if st and C.gemm_tt_supported(dy2, x2, st) and (out is None or out.is_contiguous()):
            # hand-written transposed-read MFMA GEMM (csrc/gemm.hip); the split-K reduction writes
            # the gradient-bucket slot directly when one is given
            return C.gemm_tt(dy2, x2, st, dy2.dtype, out=out)
    if s == 1 or not (dy2.is_contiguous() and x2.is_contiguous()):
        return torch.mm(dy2.t(), x2, out=out) if out is not None else torch.mm(dy2.t(), x2)
    slabs = torch.bmm(dy2.view(s, M // s, N).transpose(1, 2), x2.view(s, M // s, K), out_dtype=torch.float32)
    return _ext.require().splitk_reduce(slabs, dy2.dtype, out)


# ---------------------------------------------------------------------------
def attention_qkv_packed(qkv, attn_bias=None, dropout_p=0.0, causal=False, scale=None, k_lens=None):
    """qkv: [B, S, 3, h, d] -> context [B, S, h, d]."""
    from ..contrib.multihead_attn import attention as _attn

    return _attn.attention_packed(qkv, attn_bias, dropout_p, causal, scale, k_lens)


def softmax_cross_entropy(logits, labels, ignore_index=-100, smoothing=0.0, reduction="mean"):
    """Cross entropy with fp32 softmax statistics (apex.contrib.xentropy semantics)."""
    from ..contrib.xentropy import softmax_xentropy

    return softmax_xentropy(logits, labels, smoothing, ignore_index, reduction)


# ---------------------------------------------------------------------------
class _FusedDense(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        from . import gemm as G

        x2 = _2d(x)
        ctx.f8 = G.fp8_state()
        y = G.linear(x2, w, b, f8=ctx.f8)
        ctx.save_for_backward(x2, w)
        ctx.params = (w, b)
        ctx.has_b = b is not None
        ctx.bdtype = b.dtype if b is not None else None
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = _2d(dy).contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            from . import gemm as G

            dx = G.dgrad(dy2, w, f8=ctx.f8).view(*dy.shape[:-1], w.shape[1])
        if ctx.needs_input_grad[1]:
            dw = _wgrad(dy2, x2, param=ctx.params[0])
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = _ext.require().colsum(dy2, ctx.bdtype, _gt(ctx.params[1]))
        return dx, dw, db


def fused_dense(x, weight, bias=None):
    if _native(x) and x.shape[-1] % 8 == 0 and weight.shape[0] % 8 == 0:
        return _FusedDense.apply(x, weight, bias)
    return F.linear(x, weight, bias)


class _DenseAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act):
        from . import gemm as G

        C = _ext.require()
        x2 = _2d(x)
        f8 = ctx.f8 = G.fp8_state()
        if act in (ACT_GELU, ACT_GELU_TANH) and b is not None and b.dtype == x2.dtype and \
                (G.use_mfma(x2, w) or f8 is not None):
            # one MFMA GEMM with bias+GELU in the epilogue; h (with bias) kept for backward
            y, h = G.linear_gelu(x2, w, b, act, f8=f8)
            ctx.save_for_backward(x2, w, h, None)
            ctx.bdtype = b.dtype
        else:
            h = torch.mm(x2, w.t())
            y = C.bias_act_fwd(h, b, act)
            ctx.save_for_backward(x2, w, h, b)
            ctx.bdtype = None
        ctx.act = act
        ctx.wparam = w
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        from . import gemm as G

        C = _ext.require()
        x2, w, h, b = ctx.saved_tensors
        if ctx.bdtype is not None:
            dh, db = C.bias_act_bwd(_2d(dy), h, None, ctx.act)
            db = C.colsum(dh, ctx.bdtype)
            b = db
        else:
            dh, db = C.bias_act_bwd(_2d(dy), h, b, ctx.act)
        dx = G.dgrad(dh, w, f8=ctx.f8).view(*dy.shape[:-1], w.shape[1]) if ctx.needs_input_grad[0] else None
        dw = _wgrad(dh, x2, param=ctx.wparam) if ctx.needs_input_grad[1] else None
        return dx, dw, (db if b is not None else None), None


def _act_ref(h, act):
    if act == ACT_GELU:
        return F.gelu(h)
    if act == ACT_GELU_TANH:
        return F.gelu(h, approximate="tanh")
    if act == ACT_RELU:
        return F.relu(h)
    return h


def dense_act(x, weight, bias, act=ACT_GELU):
    if _native(x) and weight.shape[0] % 8 == 0:
        return _DenseAct.apply(x, weight, bias, act)
    return _act_ref(F.linear(x, weight, bias), act)


def dense_gelu(x, weight, bias):
    return dense_act(x, weight, bias, ACT_GELU)


def linear_gelu(x, weight, bias):
    """gelu(x @ W^T + b) (erf GELU, as in BERT)."""
    return dense_act(x, weight, bias, ACT_GELU)


class _BiasAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, b, act):
        C = _ext.require()
        h2 = _2d(h).contiguous()
        y = C.bias_act_fwd(h2, b, act)
        ctx.save_for_backward(h2, b)
        ctx.act = act
        return y.view_as(h)

    @staticmethod
    def backward(ctx, dy):
        C = _ext.require()
        h2, b = ctx.saved_tensors
        dh, db = C.bias_act_bwd(_2d(dy), h2, b, ctx.act)
        return dh.view_as(dy), (db if b is not None else None), None


def bias_gelu(h, bias):
    if _native(h) and h.shape[-1] % 8 == 0:
        return _BiasAct.apply(h, bias, ACT_GELU)
    return F.gelu(h + bias)


# ---------------------------------------------------------------------------
class _BertEmbeddings(torch.autograd.Function):
    """y = dropout(LN(Ww[ids] + Wp[pos] + Wt[types])), pos = arange(S): one HIP kernel each way
    (csrc/fused_ops.hip embed_ln_*) instead of three gathers, two broadcast adds, LayerNorm and
    dropout; the word-table gradient is a deterministic segment sum over the id-sorted tokens (no
    atomics), the position / type / gamma / beta gradients come out of the backward kernel's
    registers as partial rows."""

    @staticmethod
    def forward(ctx, ids, tids, Ww, Wp, Wt, gamma, beta, p, eps):
        C = _ext.require()
        V, TV = Ww.shape[0], Wt.shape[0]
        # out-of-range ids are clamped (a bad gather would fault the GPU); nn.Embedding raises
        ids32 = ids.clamp(0, V - 1).to(torch.int32).contiguous()
        t32 = tids.clamp(0, TV - 1).to(torch.int32).contiguous() if tids is not None else None
        seed, off = _seed(ids.device) if p > 0 else (0, 0)
        y, sv, mean, rstd = C.embed_ln_fwd(ids32, t32, Ww, Wp, Wt, gamma, beta, float(eps), float(p), seed, off)
        ctx.save_for_backward(ids32, t32, sv, gamma, mean, rstd)
        ctx.cfg = (float(p), seed, off, V, Wp.shape[0], TV)
        ctx.params = (Ww, Wp, Wt, gamma, beta)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = _ext.require()
        ids32, t32, sv, gamma, mean, rstd = ctx.saved_tensors
        p, seed, off, V, npos, TV = ctx.cfg
        pw, pp, pt, pg, pb = ctx.params
        ds, dWp, dWt, dg, db = C.embed_ln_bwd(dy, sv, gamma, mean, rstd, t32, TV, npos, p, seed, off,
                                              dwp_out=_gt(pp), dwt_out=_gt(pt), dgamma_out=_gt(pg),
                                              dbeta_out=_gt(pb))
        sorted_ids, perm = torch.sort(ids32.view(-1), stable=True)
        dWw = C.embed_segsum(ds, sorted_ids, perm, V, _gt(pw))
        return None, None, dWw, dWp, dWt, dg, db, None, None


def bert_embeddings(input_ids, token_type_ids, word, position, token_type, gamma, beta, p=0.0, eps=1e-12,
                    training=True):
    """BERT's embedding block: dropout(LayerNorm(word[ids] + position[arange(S)] + type[types]))."""
    p = p if training else 0.0
    H = word.shape[1]
    if (_native(input_ids) and input_ids.dim() == 2 and token_type.shape[0] <= 2 and
            word.dtype in (torch.float16, torch.bfloat16) and position.dtype == word.dtype and
            token_type.dtype == word.dtype and gamma is not None and beta is not None and
            _ext.require().bdaln_supported(H) and input_ids.shape[1] <= position.shape[0]):
        return _BertEmbeddings.apply(input_ids, token_type_ids, word, position, token_type, gamma, beta, float(p),
                                     float(eps))
    S = input_ids.shape[1]
    pos = torch.arange(S, device=input_ids.device)
    x = F.embedding(input_ids, word) + F.embedding(pos, position)[None]
    if token_type_ids is not None:
        x = x + F.embedding(token_type_ids, token_type)
    else:
        x = x + token_type[0]
    x = F.layer_norm(x, (H,), gamma, beta, eps)
    return F.dropout(x, p, True) if p > 0 else x


# ---------------------------------------------------------------------------
class _DenseBDALN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, res, gamma, beta, p, eps):
        from . import gemm as G

        C = _ext.require()
        x2 = _2d(x)
        ctx.f8 = G.fp8_state()
        t = G.linear(x2, w, f8=ctx.f8)
        seed, off = _seed(x.device) if p > 0 else (0, 0)
        y, s, mean, rstd = C.bdaln_fwd(t, b, _2d(res).contiguous(), gamma, beta, float(eps), float(p),
                                       seed, off)
        ctx.save_for_backward(x2, w, s, gamma, mean, rstd)
        ctx.cfg = (p, seed, off, b is not None)
        ctx.params = (w, b, gamma, beta)
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        C = _ext.require()
        x2, w, s, gamma, mean, rstd = ctx.saved_tensors
        p, seed, off, has_b = ctx.cfg
        pw, pb, pg, pbeta = ctx.params
        dres, dt, dg, dbeta, db = C.bdaln_bwd(_2d(dy), s, gamma, mean, rstd, float(p), seed, off, has_b,
                                              dgamma_out=_gt(pg), dbeta_out=_gt(pbeta),
                                              dbias_out=_gt(pb) if has_b else None)
        from . import gemm as G

        dx = G.dgrad(dt, w, f8=ctx.f8).view(*dy.shape[:-1], w.shape[1]) if ctx.needs_input_grad[0] else None
        dw = _wgrad(dt, x2, param=pw) if ctx.needs_input_grad[1] else None
        return dx, dw, (db if has_b else None), dres.view_as(dy), dg, dbeta, None, None


def dense_bias_dropout_add_ln(x, weight, bias, residual, gamma, beta, p=0.0, eps=1e-5, training=True):
    """LayerNorm(residual + dropout(x @ W^T + b)) — BERT's post-LN sublayer output."""
    p = p if training else 0.0
    if _native(x) and _ext.require().bdaln_supported(weight.shape[0]) and gamma is not None and \
            beta is not None:
        return _DenseBDALN.apply(x, weight, bias, residual, gamma, beta, float(p), float(eps))
    t = F.linear(x, weight, bias)
    s = residual + F.dropout(t, p, True) if p > 0 else residual + t
    return F.layer_norm(s, (s.shape[-1],), gamma, beta, eps)


class _BDAPreLN(torch.autograd.Function):
    """Pre-LN residual stream step (GPT): s = res + dropout(x + b) and y = LN(s), both outputs used
    (s is the next residual, y the next sublayer's input). One bdaln kernel each way: the forward
    writes s and y in one pass (no separate LayerNorm read of s), the backward adds the residual
    stream's gradient of s (ds_extra) inside the LayerNorm backward instead of an autograd
    accumulate pass over [tokens, hidden]."""

    @staticmethod
    def forward(ctx, x, b, res, gamma, beta, p, eps):
        C = _ext.require()
        seed, off = _seed(x.device) if p > 0 else (0, 0)
        y, s, mean, rstd = C.bdaln_fwd(_2d(x).contiguous(), b, _2d(res).contiguous(), gamma, beta, float(eps),
                                       float(p), seed, off)
        ctx.save_for_backward(s, gamma, mean, rstd)
        ctx.cfg = (p, seed, off, b is not None)
        ctx.params = (b, gamma, beta)
        ctx.shape = res.shape
        return s.view(res.shape), y.view(res.shape)

    @staticmethod
    def backward(ctx, ds, dy):
        C = _ext.require()
        s, gamma, mean, rstd = ctx.saved_tensors
        p, seed, off, has_b = ctx.cfg
        pb, pg, pbeta = ctx.params
        if dy is None:
            dy = torch.zeros_like(s)
        dres, dx, dg, dbeta, db = C.bdaln_bwd(_2d(dy), s, gamma, mean, rstd, float(p), seed, off, has_b,
                                              dgamma_out=_gt(pg), dbeta_out=_gt(pbeta),
                                              dbias_out=_gt(pb) if has_b else None,
                                              ds_extra=_2d(ds) if ds is not None else None)
        return (dx.view(ctx.shape), (db if has_b else None), dres.view(ctx.shape), dg, dbeta, None, None)


def bias_dropout_add_ln(x, bias, residual, gamma, beta, p=0.0, eps=1e-5, training=True):
    """(s, LayerNorm(s)) with s = residual + dropout(x + bias): a pre-LN block's residual update fused
    with the next LayerNorm (GPT-2 / Megatron layer boundaries)."""
    p = p if training else 0.0
    if _native(x) and x.shape == residual.shape and gamma is not None and beta is not None and \
            (_ext.require().bdaln_supported(x.shape[-1]) or _ext.require().bdaln_wide_supported(x.shape[-1])):
        return _BDAPreLN.apply(x, bias, residual, gamma, beta, float(p), float(eps))
    t = x + bias if bias is not None else x
    s = residual + (F.dropout(t, p, True) if p > 0 else t)
    return s, F.layer_norm(s, (s.shape[-1],), gamma, beta, eps)


class _BiasDropoutAdd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, b, res, p):
        C = _ext.require()
        seed, off = _seed(x.device) if p > 0 else (0, 0)
        y = C.bias_dropout_add_fwd(_2d(x).contiguous(), b, _2d(res).contiguous(), float(p), seed, off)
        ctx.cfg = (p, seed, off)
        ctx.has_b = b is not None
        ctx.b_like = b
        return y.view_as(x)

    @staticmethod
    def backward(ctx, dy):
        C = _ext.require()
        p, seed, off = ctx.cfg
        tb = _gt(ctx.b_like) if ctx.has_b and ctx.needs_input_grad[1] else None
        dx, db = C.bias_dropout_add_bwd(_2d(dy), float(p), seed, off, ctx.b_like if ctx.has_b else None, tb)
        return dx.view_as(dy), (db if ctx.has_b else None), dy, None


def bias_dropout_add(x, bias, residual, p, training=True):
    """residual + dropout(x + bias) with bias grad folded into the backward kernel."""
    p = p if training else 0.0
    if _native(x) and x.shape[-1] % 8 == 0 and x.shape == residual.shape:
        return _BiasDropoutAdd.apply(x, bias, residual, float(p))
    t = x + bias if bias is not None else x
    return residual + (F.dropout(t, p, True) if p > 0 else t)


def dropout_add(x, residual, p, training=True):
    """residual + dropout(x)."""
    return bias_dropout_add(x, None, residual, p, training)
