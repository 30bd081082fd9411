"""Context parallelism: attention over a sequence sharded across a CP group.

The reference has no sequence-length parallelism at all (its only sequence mechanism is
the word LM's truncated BPTT, /root/reference/examples/word_language_model/main.py:119-124). This
module adds the two standard long-context schemes on top of the flash-attention kernels
(csrc/attention_impl.h) and torch.distributed (RCCL over xGMI on MI355X, gloo on CPU):

* ``ring_attention``: every rank keeps its query shard; the K/V shards travel around the CP ring
  (one P2P exchange per step, issued before that step's block attention so the transfer overlaps
  the kernels). Partial results are merged exactly through their log-sum-exp. Backward replays the
  ring: dQ stays home, the dK/dV partial of each K/V shard travels WITH that shard and arrives
  back at its owner after the last step. Memory is O(S_local) per rank for any ring length.
  Causal masking with the ``"zigzag"`` layout (rank r holds sequence chunks r and 2W-1-r of 2W) gives
  every rank the same amount of work per step; ``"contiguous"`` (rank r holds chunk r) idles the
  low ranks under a causal mask.
* ``ulysses_attention``: two all-to-alls swap the sharded dimension from sequence to heads
  ([B, S/W, H, D] -> [B, S, H/W, D]), attention runs on whole sequences for H/W heads, and the
  inverse all-to-all restores the sequence sharding. On the 8-GPU xGMI full mesh every peer pair
  has its own link, so all-to-all is the collective that loads all 7 links at once.

Block math: on device (bf16/fp16, head dim 32..256 after padding) each block is one
``flash_attn_fwd`` / ``flash_attn_bwd`` launch — the backward kernel is handed the MERGED output and
log-sum-exp, so its delta = rowsum(dO * O) and P = exp(s - lse) are the global ones and the block
gradients are exact. On CPU (gloo tests) the same block contract is evaluated in fp32 torch.

Dropout (``dropout_p``) draws an independent mask per (step, block) and keeps it for the backward.
"""
from __future__ import annotations

import math
import os

import torch
import torch.distributed as dist

from .. import _ext

__all__ = ["ring_attention", "ulysses_attention", "shard_sequence", "gather_sequence", "chunk_ids"]


# ----------------------------------------------------------------------------------------------
# layouts
# ----------------------------------------------------------------------------------------------
def chunk_ids(rank, world, layout):
    """Global sequence-chunk ids held by ``rank`` (in local order) and the chunk count."""
    if layout == "zigzag":
        return [rank, 2 * world - 1 - rank], 2 * world
    if layout == "contiguous":
        return [rank], world
    raise ValueError("layout must be 'zigzag' or 'contiguous', got {!r}".format(layout))


def _group_info(group):
    """(group, size, rank in group, global ranks). ``group=None``: parallel_state's CP group when
    parallel_state is initialised, otherwise no context parallelism (size 1) — even when
    torch.distributed itself is initialised."""
    if group is None:
        from . import parallel_state as ps

        group = ps.get_context_parallel_group() if ps._CONTEXT_PARALLEL_GROUP is not None else None
    if group is None:
        return None, 1, 0, [dist.get_rank() if dist.is_initialized() else 0]
    return group, dist.get_world_size(group), dist.get_rank(group), dist.get_process_group_ranks(group)


def shard_sequence(x, group=None, layout="zigzag", dim=1):
    """This rank's shard of a full sequence ``x`` (sequence along ``dim``)."""
    _, W, r, _ = _group_info(group)
    ids, n = chunk_ids(r, W, layout)
    if x.shape[dim] % n:
        raise ValueError("sequence length {} is not divisible into {} chunks".format(x.shape[dim], n))
    parts = x.chunk(n, dim=dim)
    return torch.cat([parts[i] for i in ids], dim=dim)


def gather_sequence(x, group=None, layout="zigzag", dim=1):
    """Inverse of shard_sequence: the full sequence from every rank's shard (all-gather)."""
    g, W, _, _ = _group_info(group)
    if W == 1:
        return x
    shards = [torch.empty_like(x) for _ in range(W)]
    dist.all_gather(shards, x.contiguous(), group=g)
    n = chunk_ids(0, W, layout)[1]
    full = [None] * n
    for rr, s in enumerate(shards):
        ids, _ = chunk_ids(rr, W, layout)
        for i, part in zip(ids, s.chunk(len(ids), dim=dim)):
            full[i] = part
    return torch.cat(full, dim=dim)


# ----------------------------------------------------------------------------------------------
# block attention: o, lse for one (query chunk, key chunk) pair, and its backward
# ----------------------------------------------------------------------------------------------
def _native(q):
    if not (q.is_cuda and q.dtype in (torch.bfloat16, torch.float16) and q.shape[-1] in (32, 64, 128, 256)):
        return False
    C = _ext._load()
    return C is not None and hasattr(C, "flash_attn_fwd")


def _acc_dtype(t):
    """Accumulation dtype of the torch block path and the merge: fp32, or fp64 for fp64 inputs."""
    return torch.float64 if t.dtype == torch.float64 else torch.float32


def _f(t):
    return t.to(_acc_dtype(t))


def _scores(q, k, causal, scale):
    # q [B, Sq, H, D], k [B, Sk, H, D] -> fp32 [B, H, Sq, Sk]
    s = torch.einsum("bqhd,bkhd->bhqk", _f(q), _f(k)) * scale
    if causal:
        Sq, Sk = s.shape[-2:]
        s = s.masked_fill(torch.ones(Sq, Sk, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    return s


def _blk_fwd(q, k, v, causal, scale, p):
    """(o [B, Sq, H, D] in q's dtype, lse fp32 [B, H, Sq] (natural log), aux for the backward)."""
    if _native(q):
        C = _ext.require()
        seed, offset = (0, 0)
        if p > 0:
            from ..utils.rng import philox_seed_offset

            seed, offset = philox_seed_offset(q.device)
        o, lse, dmask = C.flash_attn_fwd(q, k, v, bool(causal), float(scale), float(p), seed, offset, None, None)
        return o, lse, (seed, offset, dmask)
    s = _scores(q, k, causal, scale)
    lse = torch.logsumexp(s, dim=-1)
    pr = torch.exp(s - lse[..., None])
    keep = None
    if p > 0:
        keep = torch.rand(pr.shape, device=pr.device) >= p
        pr = pr * keep / (1.0 - p)
    o = torch.einsum("bhqk,bkhd->bqhd", pr, _f(v))
    return o.to(q.dtype), lse, keep


def _blk_bwd(do, q, k, v, o, lse, causal, scale, p, aux):
    """(dq, dk, dv) of one block given the MERGED output ``o`` and log-sum-exp ``lse`` of the rows."""
    if _native(q):
        C = _ext.require()
        seed, offset, dmask = aux
        dq = torch.empty(q.shape, dtype=q.dtype, device=q.device)
        dk = torch.empty(k.shape, dtype=k.dtype, device=k.device)
        dv = torch.empty(v.shape, dtype=v.dtype, device=v.device)
        C.flash_attn_bwd(do, q, k, v, o, lse.contiguous(), dq, dk, dv, bool(causal), float(scale), float(p), seed,
                         offset, None, dmask if p > 0 else None, None, 0, None)
        return dq, dk, dv
    s = _scores(q, k, causal, scale)
    pr = torch.exp(s - lse[..., None])
    dof, vf = _f(do), _f(v)
    delta = torch.einsum("bqhd,bqhd->bhq", dof, _f(o))
    dp = torch.einsum("bqhd,bkhd->bhqk", dof, vf)
    pd = pr
    if p > 0:
        pd = pr * aux / (1.0 - p)
        dp = dp * aux / (1.0 - p)
    dv = torch.einsum("bhqk,bqhd->bkhd", pd, dof)
    ds = pr * (dp - delta[..., None])
    dq = torch.einsum("bhqk,bkhd->bqhd", ds, _f(k)) * scale
    dk = torch.einsum("bhqk,bqhd->bkhd", ds, _f(q)) * scale
    return dq, dk, dv


def _merge(acc_o, acc_lse, o, lse, s0=0, S=None):
    """Fold one block's (o [B, Sb, H, D], lse [B, H, Sb]) into rows s0 .. s0 + Sb of the running fp32
    accumulator (acc_o [B, S, H, D], acc_lse [B, H, S]; None before the first block).

    On the GPU one HIP pass (csrc/context_parallel.hip: reads the accumulator rows and the block
    once, writes the rows once, in place — a step that sees only this rank's late chunk merges into
    that half without chunk copies); the torch composition below is the CPU / reference path."""
    S = o.shape[1] if S is None else S
    covers = s0 == 0 and o.shape[1] == S
    if _native_merge(o, lse):
        C = _ext.require()
        first = acc_o is None and covers
        if acc_o is None:
            B, _, H, D = o.shape
            if covers:
                acc_o = torch.empty(B, S, H, D, dtype=torch.float32, device=o.device)
                acc_lse = torch.empty(B, H, S, dtype=torch.float32, device=o.device)
            else:  # rows no block has reached yet: weight 0 (lse = -inf) in the merge
                acc_o = torch.zeros(B, S, H, D, dtype=torch.float32, device=o.device)
                acc_lse = torch.full((B, H, S), float("-inf"), dtype=torch.float32, device=o.device)
        C.lse_merge(acc_o, acc_lse, o, lse.contiguous(), first, s0)
        return acc_o, acc_lse
    lse = torch.where(torch.isposinf(lse), torch.full_like(lse, float("-inf")), lse)  # empty rows
    if acc_o is None:
        B, _, H, D = o.shape
        acc_o = torch.zeros(B, S, H, D, dtype=_acc_dtype(o), device=o.device)
        acc_lse = torch.full((B, H, S), float("-inf"), dtype=lse.dtype, device=o.device)
    rows = slice(s0, s0 + o.shape[1])
    a_lse = acc_lse[:, :, rows]
    new = torch.logaddexp(a_lse, lse)
    safe = torch.where(torch.isneginf(new), torch.zeros_like(new), new)
    w_old = torch.exp(a_lse - safe).transpose(1, 2).unsqueeze(-1)
    w_new = torch.exp(lse - safe).transpose(1, 2).unsqueeze(-1)
    acc_o[:, rows] = acc_o[:, rows] * w_old + _f(o) * w_new
    acc_lse[:, :, rows] = new
    return acc_o, acc_lse


def _native_merge(o, lse):
    if not (o.is_cuda and o.dtype in (torch.bfloat16, torch.float16, torch.float32) and o.dim() == 4
            and o.is_contiguous() and o.shape[-1] % 8 == 0 and o.shape[-1] <= 256 and lse.dtype == torch.float32):
        return False
    C = _ext._load()
    return C is not None and hasattr(C, "lse_merge")


def _dkv_transport_dtype(k):
    """dtype of the dK/dV partials travelling the ring: the input dtype for 16-bit inputs (each hop
    adds its fp32 block gradients into the 16-bit partial, i.e. the running sum is rounded once per
    hop — W roundings over a W-rank ring; half the P2P bytes of an fp32 partial), fp32 / fp64
    accumulation for wider inputs. APEX_CP_DKV_FP32=1 keeps 16-bit inputs' partials in fp32
    (tests/test_cp_ring_native_gpu.py bounds both against one flash call)."""
    if k.dtype in (torch.bfloat16, torch.float16) and os.environ.get("APEX_CP_DKV_FP32", "0") != "1":
        return k.dtype
    return _acc_dtype(k)


def _pairs(q_ids, k_ids, causal):
    """(qi, ki, diag) over local query chunks x source key chunks that have visible keys."""
    out = []
    for qi, a in enumerate(q_ids):
        for ki, b in enumerate(k_ids):
            if causal and b > a:
                continue
            out.append((qi, ki, causal and a == b))
    return out


def _step_calls(r, src, W, layout, causal):
    """The flash calls of one ring step: [(q_sel, k_sel, diag)] where q_sel / k_sel is a local chunk
    index or None for ALL this rank's (resp. the incoming shard's) chunks, and diag = causal mask in
    local coordinates. With the zigzag layout every step is ONE call (the pairs it replaces ran as up
    to four launches of half the size — each well under the chip's 256 CUs at Megatron shapes):
      no mask:      all queries x all keys
      causal, src == r: all queries x all keys, causal in local coordinates — [chunk r, chunk 2W-1-r]
                    on both sides, so j <= i masks exactly the invisible pairs (the late keys for
                    the early queries) and the two diagonal blocks
      src < r:      all queries x the shard's EARLY chunk (its late chunk is after both of ours)
      src > r:      our LATE chunk x all the shard's keys (our early chunk sees none of them)
    The contiguous layout keeps one (query chunk, key chunk) pair per step."""
    if layout == "zigzag":
        if not causal:
            return [(None, None, False)]
        if src == r:
            return [(None, None, True)]
        if src < r:
            return [(None, 0, False)]
        return [(1, None, False)]
    return [(qi, ki, diag) for qi, ki, diag in _pairs(*(chunk_ids(x, W, layout)[0] for x in (r, src)), causal)]


# APEX_CP_KV_SPLIT=1: a non-causal ring-step block with fewer query waves (B*H*Sq/32) than this runs
# its key range as two halves on two streams (at B*H = 20, S = 8192 over 4 ranks a step block is
# 640-1280 waves against the chip's 1024 SIMDs). Off by default: measured SLOWER
# (profiles/r4_cp_ring_emulation.jsonl: CP4 at S = 8192 144 % over one flash call with the split,
# 84 % without) — the halves' launches did not overlap enough to pay for the extra merges, dQ adds
# and stream joins of ~50-90 us blocks.
_KV_SPLIT_WAVES = 2048
_side = {}


def _kv_parts(q, k, diag):
    if diag or not _native(q) or os.environ.get("APEX_CP_KV_SPLIT", "0") != "1":
        return 1
    B, Sq, H, _ = q.shape
    waves = B * H * ((Sq + 31) // 32)
    return 2 if waves < _KV_SPLIT_WAVES and k.shape[1] >= 256 and k.shape[1] % 2 == 0 else 1


def _side_streams(device):
    key = (device.type, device.index)
    if key not in _side:
        _side[key] = [torch.cuda.Stream(device=device) for _ in range(2)]
    return _side[key]


def _on_side_streams(device, fns):
    """Run fns[i]() on side stream i (after the current stream's work), join, and return the results
    with every tensor marked as used by the current stream (the caching allocator must not hand
    their memory to the side streams while the current stream still reads it)."""
    cur = torch.cuda.current_stream(device)
    ss = _side_streams(device)
    outs = []
    for s in ss[:len(fns)]:
        s.wait_stream(cur)
    for fn, s in zip(fns, ss):
        with torch.cuda.stream(s):
            outs.append(fn())
    for s in ss[:len(fns)]:
        cur.wait_stream(s)
    for res in outs:
        for t in (res if isinstance(res, (tuple, list)) else (res,)):
            if isinstance(t, torch.Tensor) and t.is_cuda:
                t.record_stream(cur)
            elif isinstance(t, (tuple, list)):
                for u in t:
                    if isinstance(u, torch.Tensor) and u.is_cuda:
                        u.record_stream(cur)
    return outs


def _step_fwd(q, k, v, diag, scale, p):
    """[(o, lse, aux, part)] of one ring-step block: one flash call (part None), or the two key
    halves (part 0, 1) run concurrently; every entry merges into the same accumulator rows."""
    n = _kv_parts(q, k, diag)
    if n == 1:
        return [_blk_fwd(q, k, v, diag, scale, p) + (None,)]
    ks, vs = k.chunk(2, dim=1), v.chunk(2, dim=1)
    res = _on_side_streams(q.device, [lambda i=i: _blk_fwd(q, ks[i], vs[i], False, scale, p) for i in range(2)])
    return [r + (i,) for i, r in enumerate(res)]


def _step_bwd(do, q, k, v, o, lse, diag, scale, p, parts):
    """[(dq, dk, dv, part)] of one ring-step block (``parts``: its _step_fwd entries' (aux, part))."""
    if parts[0][1] is None:
        return [_blk_bwd(do, q, k, v, o, lse, diag, scale, p, parts[0][0]) + (None,)]
    ks, vs = k.chunk(2, dim=1), v.chunk(2, dim=1)
    lse = lse.contiguous()
    res = _on_side_streams(q.device, [lambda a=a, i=i: _blk_bwd(do, q, ks[i], vs[i], o, lse, False, scale, p, a)
                                      for a, i in parts])
    return [r + (i,) for r, (_, i) in zip(res, parts)]


def _rows(t, sel, n, dim):
    """Chunk ``sel`` of ``t`` along ``dim`` (``t`` itself for sel None). A view along the sequence
    dim (the flash kernels take [B, S, H, D] views with any 16-byte-aligned row strides); copied
    along other dims (the [B, H, S] log-sum-exp, read contiguous)."""
    if sel is None:
        return t
    c = t.chunk(n, dim=dim)[sel]
    return c if dim == 1 else c.contiguous()


class _Ring:
    """Async exchange with the ring neighbours (send to rank + 1, receive from rank - 1)."""

    def __init__(self, group, ranks, r):
        self.group = group
        W = len(ranks)
        self.nxt, self.prv = ranks[(r + 1) % W], ranks[(r - 1) % W]

    def start(self, tensors):
        recv = [torch.empty_like(t) for t in tensors]
        ops = [dist.P2POp(dist.isend, t, self.nxt, self.group) for t in tensors]
        ops += [dist.P2POp(dist.irecv, t, self.prv, self.group) for t in recv]
        return dist.batch_isend_irecv(ops), recv

    @staticmethod
    def finish(handle):
        reqs, recv = handle
        for q in reqs:
            q.wait()
        return recv


class _RingAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, group, ranks, r, causal, scale, p, layout):
        W = len(ranks)
        ring = _Ring(group, ranks, r)
        q_ids, _ = chunk_ids(r, W, layout)
        nq = len(q_ids)
        S = q.shape[1]
        acc_o = acc_lse = None  # fp32 [B, S, H, D] / [B, H, S] over all local query rows
        aux = {}
        cur = [k.contiguous(), v.contiguous()]
        for step in range(W):
            src = (r - step) % W
            nxt = ring.start(cur) if step < W - 1 else None  # the transfer overlaps this step's blocks
            nk = len(chunk_ids(src, W, layout)[0])
            for q_sel, k_sel, diag in _step_calls(r, src, W, layout, causal):
                blocks = _step_fwd(_rows(q, q_sel, nq, 1), _rows(cur[0], k_sel, nk, 1), _rows(cur[1], k_sel, nk, 1),
                                   diag, scale, p)
                s0 = 0 if q_sel is None else q_sel * (S // nq)
                for o, lse, _, _ in blocks:
                    acc_o, acc_lse = _merge(acc_o, acc_lse, o, lse, s0, S)
                aux[(step, q_sel, k_sel)] = [(a, part) for _, _, a, part in blocks]
            if nxt is not None:
                cur = _Ring.finish(nxt)
        out = acc_o.to(q.dtype)
        lse = acc_lse
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.cfg = (group, ranks, r, causal, scale, p, layout)
        ctx.aux = aux
        return out

    @staticmethod
    def backward(ctx, do):
        q, k, v, out, lse = ctx.saved_tensors
        group, ranks, r, causal, scale, p, layout = ctx.cfg
        W = len(ranks)
        ring = _Ring(group, ranks, r)
        q_ids, _ = chunk_ids(r, W, layout)
        nq = len(q_ids)
        do = do.contiguous()
        lse = lse.contiguous()
        dq = torch.zeros(q.shape, dtype=_acc_dtype(q), device=q.device)
        cur = [k.contiguous(), v.contiguous()]
        dkv_pending = None  # the dK/dV partial of the shard arriving with `cur`, still in flight
        for step in range(W):
            src = (r - step) % W
            nxt = ring.start(cur) if step < W - 1 else None
            nk = len(chunk_ids(src, W, layout)[0])
            grads = []
            for q_sel, k_sel, diag in _step_calls(r, src, W, layout, causal):
                gs = _step_bwd(_rows(do, q_sel, nq, 1), _rows(q, q_sel, nq, 1), _rows(cur[0], k_sel, nk, 1),
                               _rows(cur[1], k_sel, nk, 1), _rows(out, q_sel, nq, 1), _rows(lse, q_sel, nq, 2), diag,
                               scale, p, ctx.aux[(step, q_sel, k_sel)])
                for g in gs:
                    (dq if q_sel is None else dq.chunk(nq, dim=1)[q_sel]).add_(g[0])
                    grads.append((k_sel, g[3], g[1], g[2]))
            # the shard's dK/dV partial from the previous ranks (zero at step 0) + this rank's blocks
            if dkv_pending is None:
                dk_t = torch.zeros(k.shape, dtype=_dkv_transport_dtype(k), device=k.device)
                dv_t = torch.zeros(v.shape, dtype=_dkv_transport_dtype(v), device=v.device)
            else:
                dk_t, dv_t = _Ring.finish(dkv_pending)
            for k_sel, part, gk, gv in grads:
                tk = dk_t if k_sel is None else dk_t.chunk(nk, dim=1)[k_sel]
                tv = dv_t if k_sel is None else dv_t.chunk(nk, dim=1)[k_sel]
                if part is not None:  # one key half of a split block
                    tk, tv = tk.chunk(2, dim=1)[part], tv.chunk(2, dim=1)[part]
                tk.add_(gk)
                tv.add_(gv)
            if W == 1:  # no ring: the only shard is this rank's own (nothing to send to itself)
                dkv_pending = ([], [dk_t, dv_t])
                continue
            # travels with its K/V shard; after the last step this send brings it home
            dkv_pending = ring.start([dk_t, dv_t])
            if nxt is not None:
                cur = _Ring.finish(nxt)
        dk, dv = _Ring.finish(dkv_pending)
        ctx.aux = None
        return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype), None, None, None, None, None, None, None


def ring_attention(q, k, v, group=None, causal=False, scale=None, dropout_p=0.0, layout="zigzag"):
    """Attention of this rank's query shard over the whole (sharded) key sequence.

    q, k, v: [B, S_local, H, D] shards laid out by ``shard_sequence(..., layout)``; returns this
    rank's [B, S_local, H, D] output shard. ``group``: the CP group (default: parallel_state's).
    """
    g, W, r, ranks = _group_info(group)
    scale = 1.0 / math.sqrt(q.shape[-1]) if scale is None else float(scale)
    if W == 1:
        layout = "contiguous"
    if layout == "zigzag" and q.shape[1] % 2:
        raise ValueError("zigzag layout needs an even local sequence length")
    return _RingAttention.apply(q, k, v, g, ranks, r, bool(causal), scale, float(dropout_p), layout)


# ----------------------------------------------------------------------------------------------
# Ulysses: sequence <-> head all-to-all
# ----------------------------------------------------------------------------------------------
def _seq_to_head(x, group, W):
    # [B, S/W, H, D] -> [B, S, H/W, D]
    B, s, H, D = x.shape
    send = x.reshape(B, s, W, H // W, D).permute(2, 0, 1, 3, 4).contiguous()
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    return recv.permute(1, 0, 2, 3, 4).reshape(B, W * s, H // W, D)


def _head_to_seq(x, group, W):
    # [B, S, H/W, D] -> [B, S/W, H, D]
    B, S, h, D = x.shape
    send = x.reshape(B, W, S // W, h, D).permute(1, 0, 2, 3, 4).contiguous()
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    return recv.permute(1, 2, 0, 3, 4).reshape(B, S // W, W * h, D)


class _SeqToHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group, W):
        ctx.cfg = (group, W)
        return _seq_to_head(x, group, W)

    @staticmethod
    def backward(ctx, g):
        group, W = ctx.cfg
        return _head_to_seq(g.contiguous(), group, W), None, None


class _HeadToSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group, W):
        ctx.cfg = (group, W)
        return _head_to_seq(x, group, W)

    @staticmethod
    def backward(ctx, g):
        group, W = ctx.cfg
        return _seq_to_head(g.contiguous(), group, W), None, None


def ulysses_attention(q, k, v, group=None, causal=False, scale=None, dropout_p=0.0, k_lens=None):
    """DeepSpeed-Ulysses-style attention over contiguous sequence shards [B, S/W, H, D]
    (``shard_sequence(..., layout="contiguous")``); needs H % W == 0. The local attention is
    apex.contrib.multihead_attn's (flash kernels on device)."""
    from ..contrib.multihead_attn.attention import attention

    g, W, _, _ = _group_info(group)
    if W == 1:
        return attention(q, k, v, dropout_p=dropout_p, causal=causal, scale=scale, k_lens=k_lens)
    if q.shape[2] % W:
        raise ValueError("ulysses_attention needs heads ({}) divisible by the CP size ({})".format(q.shape[2], W))
    qh, kh, vh = (_SeqToHead.apply(t, g, W) for t in (q, k, v))
    scale = 1.0 / math.sqrt(q.shape[-1]) if scale is None else scale
    o = attention(qh, kh, vh, dropout_p=dropout_p, causal=causal, scale=scale, k_lens=k_lens)
    return _HeadToSeq.apply(o, g, W)
