"""Whole-sublayer autograd Functions for post-LN transformer encoders (BERT).

A post-LN encoder layer uses its input twice per sublayer — as the GEMM input and as the
residual — so autograd would sum two gradients with a separate elementwise kernel per
sublayer (two full [tokens, hidden] read-read-write passes per layer). As one Function,
the backward folds the residual gradient into the input-gradient GEMM's epilogue, and the
dense layers run on the hand-written MFMA GEMM (apex/ops/gemm.py, csrc/gemm.hip) with the
bias / GELU / dGELU(+bias grad) / residual work fused into its epilogue:

  attention sublayer: y = LN(x + dropout(Attn(x Wqkv^T + bqkv) Wo^T + bo))
      fwd: GEMM+bias -> flash attn fwd (MFMA) -> GEMM -> bias+dropout+residual+LN
      bwd: bdaln bwd -> GEMM (dctx) + split-K wgrad -> flash attn bwd -> bias colsum +
           split-K wgrad -> GEMM with the residual grad added in its epilogue
  FFN sublayer:       y = LN(x + dropout(gelu(x W1^T + b1) W2^T + b2))
      fwd: GEMM+bias+GELU (stores h and gelu(h)) -> GEMM -> bias+dropout+residual+LN
      bwd: bdaln bwd -> GEMM with dGELU(h) epilogue + bias-grad partials -> wgrads ->
           GEMM with the residual grad added in its epilogue

The numerics are those of the unfused composition in apex.ops.fused (tests compare them).
"""
from __future__ import annotations

import os

import math

import torch

from .. import _ext
from . import gemm as G
from .fused import ACT_GELU, _2d, _gt, _seed, _wgrad


# MLP forward keeps gelu'(h) for the backward (EPI_BIAS_GELU_D + EPI_MUL) by default;
# APEX_MLP_STORE=h keeps the pre-activation and re-evaluates erf/exp in the backward epilogue
_STORE_DERIV = os.environ.get("APEX_MLP_STORE", "deriv") != "h"

# Memory-efficient post-LN: the bias+dropout+residual+LN forward does not store its LN input s; the
# backward rebuilds x-hat = (y - beta) / gamma from the LN output y, which is saved anyway as the next
# sublayer's GEMM input — one [tokens, hidden] write and one saved [tokens, hidden] activation less per
# sublayer (BERT-Large b768: 80.3 -> 71 GB peak). As with any output-based LayerNorm backward, a gamma
# entry of exactly 0 makes its column's x-hat unrecoverable: a host-side check (_GammaZeroCheck, one
# batched reduction + one read per step) then has the forward allocate s too, the kernel writes it (it
# makes the same test, csrc/fused_ops.hip s_cond) and the backward reads it instead (s_alt) — exact
# gradients in every case, the extra buffer only in the degenerate one. APEX_LN_MEM=0 always stores s.
_LN_MEM = os.environ.get("APEX_LN_MEM", "1") != "0"


def _ln_mem(C, cols):
    return _LN_MEM and C.bdaln_supported(cols)


class _GammaZeroCheck:
    """Does an LN gamma hold an exact 0? Decided on the host, once per training step for all gammas.

    The s buffer of the memory-efficient mode is only needed when a gamma entry is exactly 0, and
    holding it for every sublayer until backward costs a [tokens, hidden] activation per sublayer
    (9 GB at BERT-Large b768). So the forward allocates and saves it only when this check says a
    zero is present. The check runs as ONE batched device reduction over every gamma seen so far
    plus ONE host read (a device -> host sync), the first time a sublayer runs after an optimizer
    step — every torch.optim.Optimizer step, the apex fused optimizers included (they write gammas
    through raw pointers, which no version counter sees), marks the check dirty through a global
    step post-hook — or when a gamma's version counter / storage changed (in-place writes through
    autograd-visible ops). So with gradient accumulation or a pipeline schedule the micro-batch
    forwards that follow a backward do not stall the host: one read per optimizer step. Until the
    first optimizer step of the process every backward marks it dirty too (a hand-written update
    loop through `.data`). Writes through `.data` outside an optimizer step once optimizers are in
    use, between two forwards, are not seen: that is the one case this check misses.
    """

    def __init__(self):
        self._known = {}  # id(gamma) -> (weakref, version, data_ptr, has_zero)
        self._dirty = True
        self.host_reads = 0  # device -> host reads issued (tests: one per optimizer step)
        self._steps_seen = False

    def mark_dirty(self):
        self._dirty = True

    def after_optimizer_step(self):
        self._steps_seen = True
        self._dirty = True

    def after_backward(self):
        # until an optimizer step has been seen in this process the parameters may be updated by a
        # hand-written loop (`p.data -= lr * p.grad`, invisible to version counters): re-check after
        # every backward then, as before; once the step hook has fired, only after steps
        if not self._steps_seen:
            self._dirty = True

    def has_zero(self, gamma):
        import weakref
        ent = self._known.get(id(gamma))
        if (not self._dirty and ent is not None and ent[0]() is gamma and ent[1] == gamma._version
                and ent[2] == gamma.data_ptr()):
            return ent[3]
        live = [gamma] + [e[0]() for k, e in self._known.items() if k != id(gamma)]
        live = [g for g in live if g is not None and g.device == gamma.device]
        with torch.no_grad():
            # three small launches for all gammas (cat, compare, per-gamma any) — a per-gamma
            # compare + reduce cost 96 launches / ~0.5 ms per step
            flat = torch.cat([g.reshape(-1) for g in live])
            sizes = [g.numel() for g in live]
            if len(set(sizes)) == 1:
                flags = (flat.view(len(live), -1) == 0).any(dim=1).cpu()
            else:
                flags = torch.stack([s.any() for s in (flat == 0).split(sizes)]).cpu()
        self.host_reads += 1
        self._known = {id(g): (weakref.ref(g), g._version, g.data_ptr(), bool(f)) for g, f in zip(live, flags)}
        self._dirty = False
        return self._known[id(gamma)][3]


_GZ = _GammaZeroCheck()


def _gz_after_step(opt, args, kwargs):
    _GZ.after_optimizer_step()


# every optimizer step (torch.optim and apex.optimizers alike) may have written a gamma
from torch.optim.optimizer import register_optimizer_step_post_hook  # noqa: E402

register_optimizer_step_post_hook(_gz_after_step)


def _ln_plan(C, gamma, cols, needs_grad):
    """(mem, store_s) for a bias+dropout+residual+LN forward: mem = rebuild x-hat from y in the
    backward; store_s = also keep the LN input s (mem mode: only when gamma has an exact 0)."""
    mem = _ln_mem(C, cols)
    if not mem:
        return False, True
    if not needs_grad:
        return True, False  # no backward will read it
    return True, _GZ.has_zero(gamma)


# fp8 codes written by the bias+dropout+residual+LayerNorm kernels themselves (apex.fp8 "producer-side
# quantisation"): the LN output for the next sublayer's GEMM (e4m3), dt for this sublayer's
# output-gradient GEMM (e5m2) — instead of standalone quantise passes re-reading them from HBM.
# APEX_FP8_PRODUCER=0 turns it off (A/B).
_FP8_PRODUCER = os.environ.get("APEX_FP8_PRODUCER", "1") != "0"


def _q8(f8, key, fmt, like, shape=None):
    """(codes, scale, amax, fmt, slot) for a producer kernel, or None (no fp8 / first use)."""
    if f8 is None or not _FP8_PRODUCER:
        return None
    return f8.produce(key, fmt, like, shape=shape)


def _q8_kw(q8, only=False):
    if q8 is None:
        return {}
    kw = dict(q8_out=q8[0], q8_scale=q8[1], q8_amax=q8[2], q8_fmt=q8[3])
    if only:
        kw["q8_only"] = True
    return kw


def _wgrad_f8(dy2, x2, param, f8, d8, x8, dy_only, x_only):
    """_wgrad, or _wgrad_codes_only when either operand exists as fp8 codes only."""
    if dy_only or x_only:
        return _wgrad_codes_only(None if dy_only else dy2, None if x_only else x2, param, f8, d8, x8, dy2.dtype)
    return _wgrad(dy2, x2, param=param, f8=(f8, d8, x8))


def _q8_file(f8, t, q8, key, fmt, codes_only=False):
    if f8 is None or not _FP8_PRODUCER:
        return
    if q8 is not None:
        f8.register(t, q8[0], q8[4], q8[3], codes_only=codes_only)
    else:
        f8.quantize_output(t, key, fmt)  # first use: measure with current scaling


def _wgrad_codes_only(dy2, x2, param, f8, d8, x8, dtype):
    """Weight gradient dy2^T x2 when one operand (``dy2`` or ``x2`` None) exists only as fp8 codes
    (apex.fp8 codes_only_ok): the fp8 product on the codes; where that declines (main_grad
    accumulation, a non-contiguous target, a shape the fp8 kernel rejects) the 16-bit product on the
    codes' dequantised values — the same values the fp8 product uses, never the unwritten tensor."""
    out = _gt(param) if param is not None else None
    if getattr(param, "main_grad", None) is None and (out is None or out.is_contiguous()):
        r = f8.wgrad(d8, x8, dtype, out=out)
        if r is not None:
            return r
    if dy2 is None:
        dy2 = f8.dequantize(d8, f8._bwd, dtype)
    if x2 is None:
        x2 = f8.dequantize(x8, f8._fwd, dtype)
    return _wgrad(dy2, x2, param=param)


class _AttnSublayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wqkv, bqkv, wo, bo, gamma, beta, heads, p_attn, p_hidden, eps, causal, k_lens):
        C = _ext.require()
        B, S, E = x.shape
        d = E // heads
        scale = 1.0 / math.sqrt(d)
        x2 = _2d(x)
        f8 = G.fp8_state()
        qkv = G.linear(x2, wqkv, bqkv, f8=f8)
        # fp8: the GEMMs' activation codes are kept for the weight gradients (apex.fp8 operand_codes)
        x8 = f8.operand_codes(x2) if f8 is not None else None
        q, k, v = qkv.view(B, S, 3, heads, d).unbind(2)
        sa, oa = _seed(x.device) if p_attn > 0 else (0, 0)
        # fp8: the flash forward also writes the e4m3 codes of its output, the attention-out GEMM's
        # operand (slot = that GEMM's "x" slot), instead of a standalone quantise pass over [tokens, E]
        okey = (f8.key_of(wo), "x") if f8 is not None else None
        q8o = _q8(f8, okey, f8._fwd, qkv, shape=(B, S, heads, d)) if f8 is not None else None
        o, lse, dmask = C.flash_attn_fwd(q, k, v, bool(causal), scale, float(p_attn), sa, oa, k_lens,
                                         **({} if q8o is None else dict(q8_out=q8o[0], q8_scale=q8o[1],
                                                                        q8_amax=q8o[2], q8_fmt=q8o[3])))
        o2 = o.view(B * S, E)
        if f8 is not None:
            _q8_file(f8, o2, None if q8o is None else (q8o[0].view(B * S, E),) + tuple(q8o[1:]), okey, f8._fwd)
        t = G.linear(o2, wo, f8=f8)
        ctx.f8codes = (x8, f8.operand_codes(o2) if f8 is not None else None)
        sh, oh = _seed(x.device) if p_hidden > 0 else (0, 0)
        mem, store_s = _ln_plan(C, gamma, E, any(ctx.needs_input_grad))
        ykey = (f8.key_of(gamma), "y") if f8 is not None else None
        q8 = _q8(f8, ykey, f8._fwd, t) if f8 is not None else None
        y, s, mean, rstd = C.bdaln_fwd(t, bo, x2.contiguous(), gamma, beta, float(eps), float(p_hidden), sh, oh,
                                       store_s=store_s, s_cond=mem, **_q8_kw(q8))
        if f8 is not None:
            _q8_file(f8, y, q8, ykey, f8._fwd)
        ctx.save_for_backward(x2, wqkv, qkv, o, lse, k_lens, dmask, wo, y if mem else s, gamma, mean, rstd,
                              s if mem and store_s else None)
        ctx.ln_beta = beta if mem else None
        ctx.f8 = f8
        ctx.params = (wqkv, bqkv, wo, bo, gamma, beta)
        ctx.cfg = (B, S, E, heads, d, scale, causal, p_attn, sa, oa, p_hidden, sh, oh, bqkv is not None,
                   bo is not None, bqkv.dtype if bqkv is not None else None)
        return y.view(B, S, E)

    @staticmethod
    def backward(ctx, dy):
        C = _ext.require()
        _GZ.after_backward()
        x2, wqkv, qkv, o, lse, k_lens, dmask, wo, s, gamma, mean, rstd, s_alt = ctx.saved_tensors
        B, S, E, heads, d, scale, causal, p_attn, sa, oa, p_hidden, sh, oh, has_bqkv, has_bo, bdt = ctx.cfg
        pqkv, pbqkv, pwo, pbo, pg, pb = ctx.params
        f8 = ctx.f8
        dkey = (f8.key_of(wo), "dy") if f8 is not None else None
        q8 = _q8(f8, dkey, f8._bwd, s) if f8 is not None else None
        # codes only: dt's consumers are the out-projection input-gradient GEMM and its weight gradient
        tconly = q8 is not None and f8.codes_only_ok(_2d(dy), wo, wo.shape[0], wo.shape[1])
        dres, dt, dgamma, dbeta, dbo = C.bdaln_bwd(_2d(dy), s, gamma, mean, rstd, float(p_hidden), sh, oh, has_bo,
                                                   dgamma_out=_gt(pg), dbeta_out=_gt(pb),
                                                   dbias_out=_gt(pbo) if has_bo else None, beta=ctx.ln_beta,
                                                   s_alt=s_alt, **_q8_kw(q8, tconly))
        if q8 is not None:
            f8.register(dt, q8[0], q8[4], q8[3], codes_only=tconly)
        dctx = G.dgrad(dt, wo, f8=f8).view(B, S, heads, d)
        x8, o8 = ctx.f8codes
        dt8 = f8.operand_codes(dt) if f8 is not None else None
        if tconly and dt8 is None:
            raise RuntimeError("apex.fp8: the codes-only output gradient was not consumed as fp8 codes")
        dwo = _wgrad_f8(dt, o.view(B * S, E), pwo, f8, dt8, o8, tconly, False)
        q, k, v = qkv.view(B, S, 3, heads, d).unbind(2)
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = dqkv.view(B, S, 3, heads, d).unbind(2)
        # the attention backward also emits per-sequence column sums of dq/dk/dv (the QKV bias
        # gradient before the sum over the batch) — no separate pass over dqkv
        dsum = torch.zeros(B, 3 * E, device=dqkv.device, dtype=torch.float32) if has_bqkv else None
        # fp8: the e5m2 codes of dq / dk / dv for the QKV input-gradient GEMM (its "dy" slot), written by
        # the flash backward itself where it runs as one kernel (Sk <= 128)
        qkey = (f8.key_of(wqkv), "dy") if f8 is not None else None
        q8d = _q8(f8, qkey, f8._bwd, dqkv) if f8 is not None else None
        kw = {}
        # codes only: dqkv's consumers are the QKV input-gradient GEMM (+ residual) and the QKV weight
        # gradient (the bias gradient comes from the kernel's own column sums)
        qconly = q8d is not None and f8.codes_only_ok(_2d(dy), wqkv, wqkv.shape[0], wqkv.shape[1], aux=_2d(dres))
        if q8d is not None:
            cq, ck, cv = q8d[0].view(B, S, 3, heads, d).unbind(2)
            kw = dict(q8_dq=cq, q8_dk=ck, q8_dv=cv, q8_scale=q8d[1], q8_amax=q8d[2], q8_fmt=q8d[3], q8_only=qconly)
        written = C.flash_attn_bwd(dctx, q, k, v, o, lse, dq, dk, dv, bool(causal), scale, float(p_attn), sa, oa,
                                   k_lens, dmask, dsum, **kw)
        qconly = qconly and written  # (the two-kernel backward writes no codes and stores dqkv)
        if q8d is not None and written:
            f8.register(dqkv, q8d[0], q8d[4], q8d[3], codes_only=qconly)
        dbqkv = C.partial_colsum(dsum, bdt, _gt(pbqkv)) if has_bqkv else None
        dx = G.dgrad_resid(dqkv, wqkv, dres, f8=f8)  # residual grad accumulated in the GEMM epilogue
        dq8 = f8.operand_codes(dqkv) if f8 is not None else None
        if qconly and dq8 is None:
            raise RuntimeError("apex.fp8: the codes-only attention input gradient was not consumed as fp8 codes")
        dwqkv = _wgrad_f8(dqkv, x2, pqkv, f8, dq8, x8, qconly, False)
        return (dx.view(B, S, E), dwqkv, dbqkv, dwo, dbo if has_bo else None, dgamma, dbeta,
                None, None, None, None, None, None)


class _FFNSublayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, gamma, beta, p, eps, act):
        C = _ext.require()
        x2 = _2d(x)
        f8 = ctx.f8 = G.fp8_state()
        if act == ACT_GELU and b1 is not None:
            # g = gelu(h), h = x W1^T + b1; the backward keeps gelu'(h) (computed in this epilogue
            # from the same exp/erf) rather than h. fp8: the epilogue also writes g's e4m3 codes for
            # the W2 GEMM (producer slot keyed by W1, role "y")
            gkey = (f8.key_of(w1), "y") if f8 is not None else None
            q8 = _q8(f8, gkey, f8._fwd, x2, shape=(x2.shape[0], w1.shape[0])) if f8 is not None else None
            # codes only: g's 16-bit values are not stored when its two consumers (the W2 GEMM below
            # and the W2 weight gradient) read its fp8 codes
            conly = q8 is not None and _STORE_DERIV and f8.codes_only_ok(x2, w2, w2.shape[1], w2.shape[0])
            g, h = G.linear_gelu_d(x2, w1, b1, f8=f8, q8=q8, codes_only=conly) if _STORE_DERIV else \
                G.linear_gelu(x2, w1, b1, f8=f8, q8=q8)
            x8 = f8.operand_codes(x2) if f8 is not None else None
            if f8 is not None:
                written = f8.q8_written(q8)
                conly = conly and written  # (a declined fp8 GEMM stored g in full)
                _q8_file(f8, g, q8 if written else None, gkey, f8._fwd, codes_only=conly)
            hb = None
        else:
            h = torch.mm(x2, w1.t())
            g = C.bias_act_fwd(h, b1, act)
            hb = b1
            x8 = None
            conly = False
        t = G.linear(g, w2, f8=f8)
        ctx.f8codes = (x8, f8.operand_codes(g) if f8 is not None else None)
        if conly and ctx.f8codes[1] is None:
            raise RuntimeError("apex.fp8: the codes-only MLP activation was not consumed as fp8 codes")
        ctx.g_conly = conly
        seed, off = _seed(x.device) if p > 0 else (0, 0)
        mem, store_s = _ln_plan(C, gamma, x2.shape[1], any(ctx.needs_input_grad))
        ykey = (f8.key_of(gamma), "y") if f8 is not None else None
        q8 = _q8(f8, ykey, f8._fwd, t) if f8 is not None else None
        y, s, mean, rstd = C.bdaln_fwd(t, b2, x2.contiguous(), gamma, beta, float(eps), float(p), seed, off,
                                       store_s=store_s, s_cond=mem, **_q8_kw(q8))
        if f8 is not None:
            _q8_file(f8, y, q8, ykey, f8._fwd)
        ctx.save_for_backward(x2, w1, hb, h, None if conly else g, w2, y if mem else s, gamma, mean, rstd,
                              s if mem and store_s else None)
        ctx.ln_beta = beta if mem else None
        ctx.cfg = (p, seed, off, act, b2 is not None, b1.dtype if b1 is not None else None)
        ctx.params = (w1, b1, w2, b2, gamma, beta)
        return y.view_as(x)

    @staticmethod
    def backward(ctx, dy):
        C = _ext.require()
        _GZ.after_backward()
        x2, w1, hb, h, g, w2, s, gamma, mean, rstd, s_alt = ctx.saved_tensors
        p, seed, off, act, has_b2, b1dt = ctx.cfg
        f8 = ctx.f8
        pw1, pb1, pw2, pb2, pg, pb = ctx.params
        dkey = (f8.key_of(w2), "dy") if f8 is not None else None
        q8 = _q8(f8, dkey, f8._bwd, s) if f8 is not None else None
        # codes only: dt's consumers are the W2 input-gradient GEMM (its epilogue reads gelu'(h) / h)
        # and the W2 weight gradient
        tconly = q8 is not None and f8.codes_only_ok(_2d(dy), w2, w2.shape[0], w2.shape[1],
                                                     aux=h if hb is None and act == ACT_GELU and b1dt is not None else None)
        dres, dt, dgamma, dbeta, db2 = C.bdaln_bwd(_2d(dy), s, gamma, mean, rstd, float(p), seed, off, has_b2,
                                                   dgamma_out=_gt(pg), dbeta_out=_gt(pb),
                                                   dbias_out=_gt(pb2) if has_b2 else None, beta=ctx.ln_beta,
                                                   s_alt=s_alt, **_q8_kw(q8, tconly))
        if q8 is not None:
            f8.register(dt, q8[0], q8[4], q8[3], codes_only=tconly)
        if hb is None and act == ACT_GELU and b1dt is not None:
            tb1 = _gt(pb1)
            # fp8: the epilogue also writes dh's e5m2 codes for the W1 dgrad (W1's own "dy" slot)
            hkey = (f8.key_of(w1), "dy") if f8 is not None else None
            q8h = _q8(f8, hkey, f8._bwd, dt, shape=(dt.shape[0], w1.shape[0])) if f8 is not None else None
            # codes only: dh's consumers are the W1 input-gradient GEMM (+ residual) and the W1 gradient
            dconly = q8h is not None and _STORE_DERIV and f8.codes_only_ok(dt, w1, w1.shape[0], w1.shape[1], aux=dres)
            if _STORE_DERIV:
                # (dt W2) * gelu'(h) (stored) and its column sums
                dh, db1 = G.dgrad_mul(dt, w2, h, b1dt, f8=f8, bias_grad_out=tb1, q8=q8h, codes_only=dconly)
            else:
                dh, db1 = G.dgrad_dgelu(dt, w2, h, b1dt, f8=f8, bias_grad_out=tb1, q8=q8h)  # (dt W2) * gelu'(h) from h
            dt8 = f8.operand_codes(dt) if f8 is not None else None
            if q8h is not None and f8.q8_written(q8h):
                f8.register(dh, q8h[0], q8h[4], q8h[3], codes_only=dconly)
            else:
                dconly = False
            if tb1 is not None and db1 is not None and db1.data_ptr() != tb1.data_ptr():
                db1 = tb1.copy_(db1)  # a path that could not write the slot: keep the handed-out view valid
        else:
            dh, db1 = C.bias_act_bwd(G.dgrad(dt, w2, f8=f8), h, hb, act)
            dt8 = f8.operand_codes(dt) if f8 is not None else None
            dconly = False
        x8, g8 = ctx.f8codes
        if tconly and dt8 is None:
            raise RuntimeError("apex.fp8: the codes-only output gradient was not consumed as fp8 codes")
        dw2 = _wgrad_f8(dt, g, pw2, f8, dt8, g8, tconly, ctx.g_conly)
        dx = G.dgrad_resid(dh, w1, dres, f8=f8)  # residual grad accumulated in the GEMM epilogue
        dh8 = f8.operand_codes(dh) if f8 is not None else None
        if dconly:
            if dh8 is None:
                raise RuntimeError("apex.fp8: the codes-only MLP hidden gradient was not consumed as fp8 codes")
            dw1 = _wgrad_codes_only(None, x2, pw1, f8, dh8, x8, dt.dtype)
        else:
            dw1 = _wgrad(dh, x2, param=pw1, f8=(f8, dh8, x8))
        return (dx.view_as(dy), dw1, db1 if b1dt is not None else None, dw2, db2 if has_b2 else None, dgamma,
                dbeta, None, None, None)


class _MLP(torch.autograd.Function):
    """gelu(x W1^T + b1) W2^T (the second bias is left to the caller's bias+dropout+residual
    kernel): one MFMA GEMM with bias+GELU in its epilogue, then the output GEMM; backward is
    the output-gradient GEMM with the dGELU + bias-grad epilogue, the input-gradient GEMM and
    the two weight gradients."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, act):
        x2 = _2d(x)
        f8 = ctx.f8 = G.fp8_state()
        if _STORE_DERIV:
            g, gd = G.linear_gelu_d(x2, w1, b1, act, f8=f8)  # gelu(h) and gelu'(h)
        else:
            g, gd = G.linear_gelu(x2, w1, b1, act, f8=f8)  # gelu(h) and h
        x8 = f8.operand_codes(x2) if f8 is not None else None
        t = G.linear(g, w2, f8=f8)
        ctx.f8codes = (x8, f8.operand_codes(g) if f8 is not None else None)
        ctx.save_for_backward(x2, w1, gd, g, w2)
        ctx.params = (w1, b1, w2)
        ctx.act = act
        ctx.b1dt = b1.dtype
        return t.view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dt):
        x2, w1, gd, g, w2 = ctx.saved_tensors
        pw1, pb1, pw2 = ctx.params
        dt2 = _2d(dt).contiguous()
        tb1 = _gt(pb1)
        if _STORE_DERIV:
            dh, db1 = G.dgrad_mul(dt2, w2, gd, ctx.b1dt, f8=ctx.f8, bias_grad_out=tb1)
        else:
            dh, db1 = G.dgrad_dgelu(dt2, w2, gd, ctx.b1dt, act=ctx.act, f8=ctx.f8, bias_grad_out=tb1)
        f8 = ctx.f8
        dt8 = f8.operand_codes(dt2) if f8 is not None else None
        if tb1 is not None and db1 is not None and db1.data_ptr() != tb1.data_ptr():
            db1 = tb1.copy_(db1)
        x8, g8 = ctx.f8codes
        dw2 = _wgrad(dt2, g, param=pw2, f8=(f8, dt8, g8))
        dx = G.dgrad(dh, w1, f8=f8).view(*dt.shape[:-1], w1.shape[1])
        dw1 = _wgrad(dh, x2, param=pw1, f8=(f8, f8.operand_codes(dh) if f8 is not None else None, x8))
        return dx, dw1, db1, dw2, None


def mlp(x, w1, b1, w2, act=ACT_GELU):
    """gelu(x W1^T + b1) W2^T for GELU (act 0) / tanh-GELU (act 1) MLPs; None when the fused
    path does not apply (caller composes the ops)."""
    if not (_ext.use_native(x) and x.dtype in (torch.float16, torch.bfloat16) and b1 is not None and
            act in (0, 1) and w1.dtype == x.dtype and w2.dtype == x.dtype and b1.dtype == x.dtype):
        return None
    return _MLP.apply(x, w1, b1, w2, int(act))


def _ok(x, *dims):
    return _ext.use_native(x) and x.dtype in (torch.float16, torch.bfloat16) and x.is_contiguous() and \
        all(d % 8 == 0 for d in dims) and _ext.require().bdaln_supported(x.shape[-1])


def attention_sublayer(x, wqkv, bqkv, wo, bo, gamma, beta, heads, p_attn=0.0, p_hidden=0.0, eps=1e-12,
                       causal=False, k_lens=None, training=True):
    """LN(x + dropout(MHA(x) Wo^T + bo)) for x [B, S, E]; returns None when the fused path does
    not apply (caller falls back to the op-by-op composition)."""
    E = x.shape[-1]
    d = E // heads
    if not (_ok(x, E) and d in (32, 64, 128, 256) and gamma is not None and beta is not None):
        return None
    p_attn = p_attn if training else 0.0
    p_hidden = p_hidden if training else 0.0
    return _AttnSublayer.apply(x, wqkv, bqkv, wo, bo, gamma, beta, int(heads), float(p_attn), float(p_hidden),
                               float(eps), bool(causal), k_lens)


def ffn_sublayer(x, w1, b1, w2, b2, gamma, beta, p=0.0, eps=1e-12, act=ACT_GELU, training=True):
    """LN(x + dropout(act(x W1^T + b1) W2^T + b2)); None when the fused path does not apply."""
    if not (_ok(x, x.shape[-1], w1.shape[0]) and gamma is not None and beta is not None):
        return None
    return _FFNSublayer.apply(x, w1, b1, w2, b2, gamma, beta, float(p if training else 0.0), float(eps), int(act))
