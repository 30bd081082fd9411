"""FP8 training for the dense GEMMs: per-tensor scaled OCP e4m3 / e5m2 on gfx950's block-scaled
MFMA (``v_mfma_scale_f32_16x16x128_f8f6f4``, csrc/gemm.hip fp8 instantiation) — about 2x the
bf16 MFMA rate on MI355X (tools/fp8_gemm_bench.py, profiles/r2_fp8_gemm.jsonl).

The reference (apex) has no fp8 path; this is an MI355X-first extension of its amp O2 flow.

What runs in fp8
  forward   y = x W^T (+ bias / GELU / residual epilogue)    x: e4m3, W: e4m3
  backward  dx = dy W (+ dGELU / residual epilogue)          dy: e5m2 ("hybrid"), W^T: e4m3
  weight    dW = dy^T x                                        dy: e5m2, x: e4m3 (the SAME codes the
            two GEMMs above consumed, kept from the forward; csrc/gemm.hip gemm_tt_f8, a
            ds_read_b64_tr_b8 transposed-read main loop over the token-major codes, fp32 split-K
            slabs rounded once into the gradient slot). Recipe ``fp8_wgrad`` / APEX_FP8_WGRAD=0:
            bf16 weight gradients instead.
  Attention, normalisation and the optimizer stay in the activation dtype. Outputs are bf16 /
  fp16, produced by the same fused epilogues as the bf16 path.

Scaling
  * weights: current scaling — quantised (and transposed for the backward) once per optimizer
    step from their exact amax, cached until the next ``step()``;
  * activations and gradients: delayed scaling — each quantisation records max|x| on the device
    (inside the quantise kernel); ``step()`` folds those into an ``amax_history_len`` window and
    recomputes every scale (``scale = fmt_max * 2^-margin / max(window)``) in ONE kernel launch,
    with an optional MAX all-reduce of the step's amaxes over ``amax_reduction_group`` (one
    small RCCL call per step). A tensor's first quantisation uses current scaling.
  Nothing here synchronises with the host.

Producer-side quantisation
  The post-LN blocks (apex.ops.blocks) have their bias+dropout+residual+LayerNorm kernels write
  the fp8 codes of their output next to the bf16 value: the LN output (e4m3, the next sublayer's
  GEMM operand; slot keyed by the LN's gamma, role "y") and, in backward, dt (e5m2 under the
  consuming GEMM's own "dy" slot). ``produce()`` hands the kernel its scale / amax and an output
  buffer; ``register()`` files the codes under the bf16 tensor; the consuming ``forward_gemm`` /
  ``backward_gemm`` takes them instead of running a standalone quantise pass over that tensor.
  Codes only (``codes_only_ok``, APEX_FP8_CODES_ONLY=0 turns it off): where every consumer of a
  producer's output reads codes — the MLP's gelu(H) and dH (fp8 GEMM epilogues), the sublayers'
  output gradient dt (LayerNorm backward) and the attention input gradient dQKV (flash backward) —
  the 16-bit output is not stored at all. A weight gradient that still has to run in 16 bits takes
  the codes' dequantised values. Measured on the BERT-Large step: 152.5 -> 144.2 ms (1.22x ->
  1.29x bf16), peak memory 108.8 -> 90.8 GB (profiles/r6_bench_fp8_codes_only_ab.jsonl).

Use
  amp:       ``amp.initialize(model, opt, opt_level="O2", fp8=True)`` (or an ``Fp8Recipe``) — the
             patched ``optimizer.step()`` calls ``apex.fp8.step()``;
  explicit:  ``with apex.fp8.fp8_autocast(recipe=Fp8Recipe()): loss = model(x)``; call
             ``apex.fp8.step()`` after each optimizer step.
  Which layers: the fused transformer blocks and dense ops of apex.ops (BERT / GPT / Megatron
  model zoo, FusedDense, MLP) whenever their shapes fit the fp8 kernel (contraction % 128,
  output width % 8, bf16/fp16 activations); others stay bf16.
"""
from __future__ import annotations

import contextlib
import dataclasses
import os
import weakref
from typing import Optional

import torch

E4M3, E5M2 = 0, 1
FMT_MAX = {E4M3: 448.0, E5M2: 57344.0}
_FMT_NAMES = {"e4m3": E4M3, "e5m2": E5M2}

__all__ = ["Fp8Recipe", "Fp8State", "fp8_autocast", "enable", "disable", "active", "step", "state",
           "E4M3", "E5M2", "FMT_MAX"]


@dataclasses.dataclass
class Fp8Recipe:
    """Delayed-scaling recipe. ``fwd_format`` for activations and weights, ``bwd_format`` for
    output gradients ("hybrid" = e4m3 forward, e5m2 backward, the default)."""

    margin: int = 0
    amax_history_len: int = 16
    fwd_format: str = "e4m3"
    bwd_format: str = "e5m2"
    amax_reduction_group: Optional[object] = None
    reduce_amax: bool = True
    fp8_wgrad: bool = True

    def fmt(self, which):
        name = self.fwd_format if which == "fwd" else self.bwd_format
        if name not in _FMT_NAMES:
            raise ValueError(f"fp8 format {name!r}: expected 'e4m3' or 'e5m2'")
        return _FMT_NAMES[name]


def _C():
    from .. import _ext

    return _ext.require()


# fp8 weight gradients: "auto" (slice policy below), "0" (bf16 weight gradients), or a slice count
_FP8_WGRAD = os.environ.get("APEX_FP8_WGRAD", "auto")
# batched per-step weight quantisation (Fp8State._batch_weights); "0": one weight at a time
_FP8_WBATCH = os.environ.get("APEX_FP8_WBATCH", "1")
# codes-only producer outputs (Fp8State.codes_only_ok); "0": the 16-bit outputs are always stored
_FP8_CODES_ONLY = os.environ.get("APEX_FP8_CODES_ONLY", "1")


def _f8_wgrad_splits(R, P, Q, cus=256):
    """Split-K slices for the fp8 weight gradient dW [P, Q] over R tokens. With t 256x256 output
    tiles and s slices the kernel runs ceil(t s / CUs) workgroup rounds of R / s tokens each, so
    pick the s in {1, 2, 4, 8, 16} minimising ceil(t s / CUs) / s (ties: fewer slices, less fp32
    slab traffic), each slice a whole number of 128-token K-tiles and >= 1024 tokens long.
    Measured at BERT-Large's 98304 tokens (tools/wgrad_f8_bench.py, profiles/r5_wgrad_f8.jsonl):
    QKV (48 tiles) 381 us at 16 slices vs 402 / 414 at 4 / 8; out-projection (16) 130 at 16 vs 202
    at 8; FFN (64) 442 / 431 at 4 vs 465-532 at 8 / 16 — the model's picks."""
    if _FP8_WGRAD not in ("auto", "", "0"):
        s = int(_FP8_WGRAD)
        return s if R % (128 * s) == 0 else 0
    tiles = -(-P // 256) * -(-Q // 256)
    best, best_cost = 1, None
    for s in (1, 2, 4, 8, 16):
        if R % (128 * s) or (s > 1 and R // s < 1024):
            break
        cost = -(-tiles * s // cus) / s
        if best_cost is None or cost < best_cost - 1e-12:
            best, best_cost = s, cost
    return best


class Fp8State:
    """Scaling metadata for every quantised tensor role, in device buffers indexed by slot:
    ``hist [cap, L]``, ``amax [cap]`` (this step's running max), ``scale``, ``scale_inv``,
    ``fmax``. Slots are keyed by (weight, role) with role in {"w", "x", "dy"}."""

    def __init__(self, recipe: Fp8Recipe | None = None, device=None):
        self.recipe = recipe or Fp8Recipe()
        self._next_key = 0
        self._free: list = []  # slot indices released by dead tensors, reused lowest first
        self._dying: list = []  # released since the last step(); moved to _free (sorted) at step()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.smax_scale = 2.0 ** (-self.recipe.margin)
        self._cap = 0
        self.n = 0
        self.idx = 0
        self.gen = 0
        self.steps = 0
        self.slots: dict = {}
        self._fresh: set = set()
        self._wcache: dict = {}
        # the previous step's weights (key -> (weakref, slot, W^T used)): the first weight request of
        # a step quantises all of them in one batched pass (_batch_weights)
        self._wprev: dict = {}
        self._fwd = self.recipe.fmt("fwd")
        self._bwd = self.recipe.fmt("bwd")
        # (data_ptr, numel) -> (weakref to the tensor, version, codes, slot, fmt): producer-made codes
        # awaiting their consuming GEMM. The tensor itself is NOT kept alive (an output nobody
        # consumes — the last layer's y, eval loops without step() — would otherwise stay pinned);
        # while the weakref is alive the (pointer, numel) key cannot name recycled memory.
        self._pre: dict = {}
        self._pre_bytes = 0
        # (data_ptr, numel) -> weakref: outputs whose 16-bit values were never stored (codes only)
        self._conly: dict = {}
        self.prequant_hits = 0
        # (operand, its _version, codes, scale_inv) of the last fp8 GEMM's activation operand
        self._last = None
        self.wgrad_calls = 0  # fp8 weight-gradient GEMMs run (tests: the fp8 kernel, not the bf16 fallback)
        self._grow(128)

    # ------------------------------------------------------------------ slots
    def _grow(self, cap):
        L = self.recipe.amax_history_len
        dev = self.device
        new = dict(hist=torch.zeros(cap, L, device=dev), amax=torch.zeros(cap, device=dev),
                   scale=torch.ones(cap, device=dev), scale_inv=torch.ones(cap, device=dev),
                   fmax=torch.ones(cap, device=dev))
        if self._cap:
            for k, t in new.items():
                t[: self._cap].copy_(getattr(self, k))
        for k, t in new.items():
            setattr(self, k, t)
        self._cap = cap

    def key_of(self, w) -> int:
        """Stable slot key of a weight tensor: a counter stored on the tensor at first sight (not
        ``id(w)``, which CPython recycles — a new tensor would inherit a dead one's scale history).
        When the tensor dies its slots return to a free list; replicas that run the same forward
        allocate and release in the same order, so slot i is the same role on every rank of the
        amax reduction group. A weight re-created every step (an O1 cast) thus reuses its slots
        instead of growing the buffers without bound."""
        k = getattr(w, "_apex_fp8_key", None)
        if k is None or k[0] is not self:
            k = (self, self._next_key)
            self._next_key += 1
            w._apex_fp8_key = k
            weakref.finalize(w, Fp8State._release, weakref.ref(self), k[1])
        return k[1]

    @staticmethod
    def _release(ref, key):
        st = ref()
        if st is None:
            return
        for role in ("w", "x", "dy", "y"):
            s = st.slots.pop((key, role), None)
            if s is not None:
                st._fresh.discard(s)
                # reusable only from the next step() on, in sorted order. That makes the ORDER of
                # reuse the same on every rank of the amax reduction group, not its TIMING: a tensor
                # freed by refcounting dies at the same point of the step everywhere, but one caught
                # in a reference cycle dies when the cyclic GC runs, which can fall on different
                # sides of a step() boundary on different ranks — the slot is then recycled a step
                # apart and, for that step, the reduced amax mixes two roles (a one-step scale error,
                # not a crash). Keep fp8 weights out of reference cycles to stay exact.
                st._dying.append(s)
        st._wcache.pop(key, None)
        st._wprev.pop(key, None)

    def slot(self, key, fmt) -> int:
        s = self.slots.get(key)
        if s is None:
            if self._free:
                self._free.sort()
                s = self._free.pop(0)
                self.hist[s].zero_()
                self.amax[s] = 0.0
                self.scale[s] = 1.0
                self.scale_inv[s] = 1.0
            else:
                if self.n == self._cap:
                    self._grow(2 * self._cap)
                s = self.n
                self.n += 1
            self.slots[key] = s
            self.fmax[s] = FMT_MAX[fmt]
            self._fresh.add(s)
        return s

    def _view(self, name, s):
        return getattr(self, name)[s:s + 1]

    # ------------------------------------------------------------------ quantisers
    def _current(self, x, s, fmt, transpose=False):
        """Current scaling: exact amax of x, then quantise with smax / amax (scale written)."""
        C = _C()
        am = self._view("amax", s)
        am.zero_()
        C.fp8_amax(x, am)
        q = C.fp8_quantize_t if transpose else C.fp8_quantize
        return q(x, fmt, self._view("scale", s), None, am, self._view("scale_inv", s),
                 FMT_MAX[fmt] * self.smax_scale)

    def quantize(self, x, key, fmt):
        """Delayed-scaled quantisation of an activation / gradient -> (codes uint8, scale_inv view)."""
        C = _C()
        x = x if x.is_contiguous() else x.contiguous()
        s = self.slot(key, fmt)
        if s in self._fresh:
            self._fresh.discard(s)
            y = self._current(x, s, fmt)  # amax stays recorded for the next update
        else:
            y = C.fp8_quantize(x, fmt, self._view("scale", s), self._view("amax", s))
        return y, self._view("scale_inv", s)

    def _weight_entry(self, w):
        k = self.key_of(w)
        e = self._wcache.get(k)
        if e is not None and e[0]() is w and e[1] == self.gen:
            return e
        if self._wprev:
            self._batch_weights()
            e = self._wcache.get(k)
            if e is not None and e[0]() is w and e[1] == self.gen:
                return e
        s = self.slot((k, "w"), self._fwd)
        self._fresh.discard(s)
        w8 = self._current(w.detach().contiguous(), s, self._fwd)
        e = [weakref.ref(w), self.gen, s, w8, None]
        self._wcache[k] = e
        return e

    def _batch_weights(self):
        """Quantise every weight the previous step used (and that is still alive) in one batched pass
        (csrc/fp8.hip fp8_quantize_weights: one amax and one quantise launch for all of them,
        each tile read once for the codes of W and, where the previous step needed them, W^T)
        instead of three launches per weight. Same current scaling and rounding as _current +
        weight_t. APEX_FP8_WBATCH=0: per-weight launches (A/B)."""
        prev, self._wprev = self._wprev, {}
        if _FP8_WBATCH == "0":
            return
        groups: dict = {}
        for k, (ref, slot, want_t) in prev.items():
            w = ref()
            if w is None or w.dim() != 2 or not w.is_cuda or not w.is_contiguous():
                continue
            if w.dtype not in (torch.bfloat16, torch.float16, torch.float32):
                continue
            if self.slots.get((k, "w")) != slot:
                continue
            groups.setdefault(w.dtype, []).append((k, w, slot, want_t))
        C = _C()
        smax = FMT_MAX[self._fwd] * self.smax_scale
        for items in groups.values():
            outs = C.fp8_quantize_weights([w.detach() for _, w, _, _ in items], [s for _, _, s, _ in items],
                                          [t for _, _, _, t in items], self._fwd, self.scale, self.scale_inv,
                                          self.amax, smax)
            for i, (k, w, slot, want_t) in enumerate(items):
                self._fresh.discard(slot)
                self._wcache[k] = [weakref.ref(w), self.gen, slot, outs[2 * i], outs[2 * i + 1] if want_t else None]

    def weight(self, w):
        """W [N, K] -> (e4m3 codes [N, K], scale_inv), cached for this optimizer step."""
        e = self._weight_entry(w)
        return e[3], self._view("scale_inv", e[2])

    def weight_t(self, w):
        """W^T [K, N] codes (same scale as ``weight``), cached for this optimizer step."""
        e = self._weight_entry(w)
        if e[4] is None:
            e[4] = _C().fp8_quantize_t(w.detach().contiguous(), self._fwd, self._view("scale", e[2]))
        return e[4], self._view("scale_inv", e[2])

    # ------------------------------------------------------------------ producer-side codes
    _PRE_MAX = 64  # pending entries kept at most (an unconsumed output is dropped oldest first)
    _PRE_MAX_BYTES = 4 << 30  # and at most this many bytes of pending codes

    def produce(self, key, fmt, like, shape=None):
        """Arguments for a producer kernel that writes fp8 codes of its own output ``like``:
        ``(codes_out, scale, amax, fmt, slot)`` — or None on the slot's first use, when there is
        no amax history to scale with yet (the caller then runs without the side output and
        ``quantize_output`` measures the tensor with current scaling)."""
        if not (like.is_cuda and like.dtype in (torch.bfloat16, torch.float16)):
            return None
        s = self.slot(key, fmt)
        if s in self._fresh:
            return None
        codes = torch.empty(like.shape if shape is None else shape, dtype=torch.uint8, device=like.device)
        return codes, self._view("scale", s), self._view("amax", s), fmt, s

    def register(self, t, codes, slot, fmt, codes_only=False):
        """File producer-made codes of ``t`` (format ``fmt``, scaled by ``slot``) for the GEMM that
        consumes ``t`` next. ``codes_only``: ``t``'s own values were never written (codes_only_ok)."""
        if codes_only:
            self._conly[(t.data_ptr(), t.numel())] = weakref.ref(t)
        # prune entries whose tensor died unconsumed, then cap by count and bytes (oldest first)
        for k in [k for k, e in self._pre.items() if e[0]() is None]:
            self._drop_pre(k)
        nb = codes.numel()
        while self._pre and (len(self._pre) >= self._PRE_MAX or self._pre_bytes + nb > self._PRE_MAX_BYTES):
            self._drop_pre(next(iter(self._pre)))
        key = (t.data_ptr(), t.numel())
        self._drop_pre(key)
        self._pre[key] = (weakref.ref(t), t._version, codes, slot, fmt)
        self._pre_bytes += nb

    def _recycle_slots(self):
        """Slots of tensors that died since the last step become reusable (lowest first)."""
        if self._dying:
            self._free.extend(self._dying)
            self._free.sort()
            self._dying = []

    def _drop_pre(self, key):
        e = self._pre.pop(key, None)
        if e is not None:
            self._pre_bytes -= e[2].numel()
        return e

    def quantize_output(self, t, key, fmt):
        """First use of a producer slot: standalone current-scaled quantisation of ``t`` (records
        the amax the slot's later fused passes scale with), filed like a producer's codes."""
        if not (t.is_cuda and t.dtype in (torch.bfloat16, torch.float16) and t.is_contiguous()):
            return
        s = self.slot(key, fmt)
        codes, _ = self.quantize(t, key, fmt)
        self.register(t, codes, s, fmt)

    def _is_codes_only(self, a):
        r = self._conly.get((a.data_ptr(), a.numel()))
        return r is not None and r() is not None

    def _take(self, a, fmt):
        e = self._drop_pre((a.data_ptr(), a.numel()))
        if e is None:
            if self._conly and self._is_codes_only(a):
                raise RuntimeError("apex.fp8: a codes-only output reached a GEMM without its codes")
            return None
        ref, ver, codes, s, cfmt = e
        t = ref()
        if t is None or a._version != ver or a.dtype != t.dtype or not a.is_contiguous() or cfmt != fmt:
            return None
        self.prequant_hits += 1
        return codes.view(a.shape), self._view("scale_inv", s)

    # ------------------------------------------------------------------ GEMMs
    @staticmethod
    def _fits(a, w, bias, aux, contraction, width):
        if not (a.is_cuda and a.dtype in (torch.bfloat16, torch.float16) and a.dim() == 2):
            return False
        if contraction % 128 or width % 8 or w.dim() != 2:
            return False
        if bias is not None and bias.dtype != a.dtype:
            return False
        if aux is not None and (aux.dtype != a.dtype or not aux.is_contiguous()):
            return False
        return True

    def forward_gemm(self, a, w, epi, bias=None, aux=None, q8=None, codes_only=False):
        """a [M, K] @ w[N, K]^T with epilogue ``epi`` on the fp8 kernel -> (out, extra) or None.
        ``q8`` (from ``produce``; bias+GELU epilogues): the epilogue also writes the output's fp8
        codes — ``q8_written(q8)`` tells the caller whether this call ran and wrote them.
        ``codes_only`` (with ``q8``): ``out`` is allocated but its values are not stored (the caller
        checked codes_only_ok for every consumer)."""
        if not self._fits(a, w, bias, aux, w.shape[1], w.shape[0]):
            self._last = None  # a declined GEMM must not leave an older operand's codes claimable
            return None
        pre = self._take(a, self._fwd) if self._pre or self._conly else None
        a8, ia = pre if pre is not None else self.quantize(a, (self.key_of(w), "x"), self._fwd)
        self._last = self._remember(a, a8, ia)
        w8, iw = self.weight(w)
        kw = {}
        if q8 is not None:
            kw = dict(q8_out=q8[0], q8_scale=q8[1], q8_amax=q8[2], q8_fmt=q8[3], q8_only=bool(codes_only))
            self._q8_last = q8[0]
        return _C().gemm_f8(a8, w8, ia, iw, self._fwd, epi, bias, aux, None, a.dtype, **kw)

    def q8_written(self, q8):
        """True when the last ``forward_gemm`` given ``q8`` ran on the fp8 kernel (codes written)."""
        ok = q8 is not None and getattr(self, "_q8_last", None) is q8[0]
        self._q8_last = None
        return ok

    def backward_gemm(self, dy, w, epi, aux=None, bias_grad_dtype=None, q8=None, codes_only=False):
        """dy [M, N] @ w[N, K] with epilogue ``epi`` (dy e5m2 x W^T e4m3) -> (out, extra) or None."""
        if not self._fits(dy, w, None, aux, w.shape[0], w.shape[1]):
            self._last = None
            return None
        pre = self._take(dy, self._bwd) if self._pre or self._conly else None
        d8, id_ = pre if pre is not None else self.quantize(dy, (self.key_of(w), "dy"), self._bwd)
        self._last = self._remember(dy, d8, id_)
        wt8, iw = self.weight_t(w)
        kw = {}
        if q8 is not None:  # (dGELU / MUL epilogues: the hidden gradient's codes for the W1 dgrad)
            kw = dict(q8_out=q8[0], q8_scale=q8[1], q8_amax=q8[2], q8_fmt=q8[3], q8_only=bool(codes_only))
            self._q8_last = q8[0]
        return _C().gemm_f8(d8, wt8, id_, iw, self._bwd, epi, None, aux, bias_grad_dtype, dy.dtype, **kw)

    # ------------------------------------------------------------------ weight gradients
    def operand_codes(self, a):
        """(codes, scale_inv) of ``a`` if the last ``forward_gemm`` / ``backward_gemm`` consumed it
        in fp8, else None. The fused blocks keep them for the weight gradient (``wgrad``): the
        layer input's codes from the forward, the output gradient's from the input-gradient GEMM
        — no second quantisation of either tensor. scale_inv is a view of the slot, which only
        ``step()`` rewrites, i.e. after every backward of the step."""
        e, self._last = self._last, None
        if e is None or not self.wgrad_enabled():
            return None
        t, ver, codes, sinv = e
        # the consumed operand is held (strongly: callers pass fresh reshaped views, so object identity
        # says nothing) until this claim or the next fp8 GEMM, so its memory cannot have been freed and
        # reused by another tensor; same address + shape = the same bytes, and its version counter
        # (shared by every view of the storage) rules out an in-place write since the codes were taken
        if a.data_ptr() != t.data_ptr() or tuple(a.shape) != tuple(t.shape) or t._version != ver:
            return None
        return codes, sinv

    @staticmethod
    def _remember(t, codes, sinv):
        return (t, t._version, codes, sinv)

    def wgrad_enabled(self):
        return self.recipe.fp8_wgrad and _FP8_WGRAD != "0" and self._fwd == E4M3

    # ------------------------------------------------------------------ codes-only outputs
    def codes_only_ok(self, a_like, w, contraction, width, aux=None):
        """May a producer skip storing its 16-bit output? Yes when that output's consumers all read
        fp8 codes: the next GEMM (an ``a_like``-typed operand against ``w``, given contraction /
        output width, optional ``aux``) fits the fp8 kernel, and the weight gradient that keeps the
        operand runs on its codes (fp8 weight gradients on). The fused MLP uses it for gelu(H) (the
        bias+GELU+derivative forward feeds only the W2 GEMM and the W2 gradient) and for dH (the
        multiply backward feeds only the W1 input-gradient GEMM and the W1 gradient): one [tokens,
        4 x hidden] 16-bit store less each (csrc/gemm.hip epilogue XD bit 4). A weight gradient
        that still declines fp8 (main_grad accumulation, a declined shape) takes the codes'
        dequantised values (``dequantize``), never the unwritten tensor."""
        return (_FP8_CODES_ONLY != "0" and self.wgrad_enabled() and a_like.is_cuda
                and self._fits(a_like, w, None, aux, contraction, width))

    @staticmethod
    def dequantize(codes_sinv, fmt, dtype):
        """(codes, scale_inv) -> the values they encode, in ``dtype`` (OCP e4m3fn / e5m2)."""
        codes, sinv = codes_sinv
        f8t = torch.float8_e4m3fn if fmt == E4M3 else torch.float8_e5m2
        return (codes.view(f8t).to(torch.float32) * sinv).to(dtype)

    def wgrad(self, d, x, out_dtype, out=None):
        """dW [P, Q] = dy^T x from the codes ``d`` (dy [R, P], backward format) and ``x`` (x [R, Q],
        e4m3) on the fp8 transposed-read kernel (csrc/gemm.hip gemm_tt_f8) -> out_dtype (written
        into ``out`` when given), or None when the recipe or the shape rules it out."""
        if not self.wgrad_enabled() or d is None or x is None:
            return None
        (d8, sd), (x8, sx) = d, x
        s = _f8_wgrad_splits(d8.shape[0], d8.shape[1], x8.shape[1])
        C = _C()
        if not s or not C.gemm_tt_f8_supported(d8, x8, s):
            return None
        self.wgrad_calls += 1
        return C.gemm_tt_f8(d8, x8, sd, sx, self._bwd, self._fwd, s, out_dtype, out=out)

    # ------------------------------------------------------------------ step
    def step(self):
        """Fold this step's amaxes into the history, recompute every scale, invalidate the
        weight cache (the optimizer has changed the weights). One launch (+ one optional
        all-reduce); no host synchronisation."""
        self.gen += 1
        self.steps += 1
        self._last = None
        self._wprev = {k: (e[0], e[2], e[4] is not None) for k, e in self._wcache.items() if e[0]() is not None}
        self._wcache.clear()
        self._pre.clear()
        self._pre_bytes = 0
        self._conly.clear()
        self._recycle_slots()
        if self.n == 0:
            return
        r = self.recipe
        if r.reduce_amax and torch.distributed.is_available() and torch.distributed.is_initialized():
            g = self.reduction_group()
            if torch.distributed.get_world_size(g) > 1:
                self._reduce_amax(g)
        _C().fp8_update_scales(self.hist, self.amax, self.scale, self.scale_inv, self.fmax, self.n, self.idx,
                               self.smax_scale)
        self.idx = (self.idx + 1) % r.amax_history_len

    def reduction_group(self):
        """``recipe.amax_reduction_group``, else the data-parallel group when apex.transformer's
        model parallelism is initialised (pipeline stages hold different layers and tensor-parallel
        ranks different shards: a WORLD reduction would max unrelated slots together), else WORLD."""
        if self.recipe.amax_reduction_group is not None:
            return self.recipe.amax_reduction_group
        try:
            from ..transformer import parallel_state as ps

            if ps.model_parallel_is_initialized():
                return ps.get_data_parallel_group()
        except ImportError:  # pragma: no cover
            pass
        return None

    def _reduce_amax(self, g):
        """MAX all-reduce of this step's amaxes. During the first three steps the slot counts are
        compared first (a 2-element MAX of (n, -n); a host sync that costs nothing there): ranks
        whose slots differ would otherwise hang in, or silently cross-wire, the amax reduction."""
        n = self.n
        if self.steps <= 3:
            t = torch.tensor([float(n), -float(n)], device=self.amax.device)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX, group=g)
            hi, lo = float(t[0]), -float(t[1])
            if hi != n or lo != n:
                raise RuntimeError(f"fp8 amax reduction: slot counts differ across the group ({lo:g}..{hi:g}); "
                                   "set Fp8Recipe.amax_reduction_group to a group whose ranks run the same layers")
        torch.distributed.all_reduce(self.amax[:n], op=torch.distributed.ReduceOp.MAX, group=g)

    # ------------------------------------------------------------------ checkpoint
    def state_dict(self, model=None):
        """Scaling state by parameter name (``model`` given) — restorable in another process."""
        out = {"idx": self.idx, "steps": self.steps, "recipe": dataclasses.asdict(
            dataclasses.replace(self.recipe, amax_reduction_group=None)), "slots": {}}
        names = {getattr(p, "_apex_fp8_key", (None, None))[1]: n for n, p in model.named_parameters()
                 if getattr(p, "_apex_fp8_key", (None,))[0] is self} if model is not None else {}
        for (pid, role), s in self.slots.items():
            name = names.get(pid)
            if model is not None and name is None:
                continue
            out["slots"][f"{name if name is not None else pid}:{role}"] = {
                "hist": self.hist[s].cpu(), "scale": float(self.scale[s]), "scale_inv": float(self.scale_inv[s]),
                "fmax": float(self.fmax[s]), "fresh": s in self._fresh}
        return out

    def load_state_dict(self, sd, model):
        params = dict(model.named_parameters())
        self.idx = int(sd["idx"])
        self.steps = int(sd["steps"])
        for k, v in sd["slots"].items():
            name, role = k.rsplit(":", 1)
            if name not in params:
                continue
            fmt = E4M3 if v["fmax"] == FMT_MAX[E4M3] else E5M2
            s = self.slot((self.key_of(params[name]), role), fmt)
            self.hist[s].copy_(v["hist"])
            self.scale[s] = v["scale"]
            self.scale_inv[s] = v["scale_inv"]
            if not v["fresh"]:
                self._fresh.discard(s)
        self._wcache.clear()


# ---------------------------------------------------------------------- global switch
_STATE: Optional[Fp8State] = None
_GLOBAL = False
_DEPTH = 0


def state(recipe: Fp8Recipe | None = None, device=None) -> Fp8State:
    """The process's Fp8State (created on first use)."""
    global _STATE
    if _STATE is None:
        _STATE = Fp8State(recipe, device)
    elif recipe is not None and recipe != _STATE.recipe:
        _STATE = Fp8State(recipe, device)  # a different recipe: fresh scaling state
    return _STATE


def active() -> Optional[Fp8State]:
    """The state the fused ops should quantise with right now, or None (bf16 path)."""
    if (_GLOBAL or _DEPTH) and _STATE is not None:
        return _STATE
    return None


def enable(recipe: Fp8Recipe | None = None, device=None) -> Fp8State:
    """Turn fp8 on for every subsequent forward (what amp.initialize(fp8=...) calls)."""
    global _GLOBAL
    st = state(recipe, device)
    _GLOBAL = True
    return st


def disable():
    global _GLOBAL, _STATE
    _GLOBAL = False
    _STATE = None


def step():
    """Per-optimizer-step scale update (no-op when fp8 was never used)."""
    if _STATE is not None:
        _STATE.step()


@contextlib.contextmanager
def fp8_autocast(enabled: bool = True, recipe: Fp8Recipe | None = None, device=None):
    """Quantise the fused ops' GEMMs inside the block. The backward of a forward run here uses
    fp8 too (the choice is recorded per autograd node). Scales update at ``step()``."""
    global _DEPTH
    if not enabled:
        yield None
        return
    st = state(recipe, device)
    _DEPTH += 1
    try:
        yield st
    finally:
        _DEPTH -= 1
