"""Memory-efficient (query-blocked) attention for what the MFMA flash kernels do not take: head
dims above 256 (above 128 for fp32 inputs), ``APEX_ATTN_BACKEND=chunked`` / ``APEX_ATTN_F32=0``
A/B runs. (Rounds 1-3 also sent fp32 inputs and trainable biases here; both now run on the
kernels: csrc/attention_f32.hip, and the backward kernels' bias-gradient output.)

The reference composition materialises the whole [B, h, Sq, Sk] score tensor (and autograd keeps
the softmax AND the dropout mask for backward): O(S^2) memory, 2 GB for B*h = 64 at S = 2048 in
fp32, before the gradient copies. Here the queries are processed in blocks of ``block`` rows —
scores, softmax and the P.V product live for one block at a time — and the backward recomputes
each block's probabilities from the saved log-sum-exp (flash-attention's recomputation, on
hipBLASLt/rocBLAS GEMMs: fp32 GEMMs run on the exact f32 MFMA), so memory is O(S * block) besides
the inputs and the outputs. Dropout masks are regenerated per block from a seeded generator (the
seed comes from the device generator: ``torch.manual_seed`` reproducible). The bias gradient is
the score gradient dS of every block, reduced over the bias's broadcast dimensions.

Statistics are fp32 whatever the input dtype; the output is in the input dtype.
"""
from __future__ import annotations

import math

import torch


def _block_rows(B, H, Sq, Sk, budget_bytes=64 << 20, short_rows=1024, short_budget=2 << 30):
    """Query rows per block. Training-length sequences (Sq <= ``short_rows``) run as ONE block —
    no Python loop of ~15 torch ops per block forward and backward — whenever their fp32
    temporaries fit ``short_budget`` (2 GiB, small next to 288 GB of HBM; B*H = 4096 at S = 128 is
    1 GiB). Round 3 used the 64 MB long-sequence budget everywhere, which cut the fp32 BERT-Large
    step into 16-row blocks (8 iterations x 24 layers x 3 micro-batches, fwd + bwd) and slowed it
    from 1567 to 2458 ms. Longer sequences keep O(S * block) memory: power-of-two blocks of at
    least 16 rows within ``budget_bytes``."""
    per_row = max(1, B * H * Sk * 4 * 4)  # ~4 fp32 [B, H, rows, Sk] temporaries alive per block
    if Sq <= short_rows and per_row * Sq <= short_budget:
        return int(Sq)
    rows = max(16, budget_bytes // per_row)
    return int(min(Sq, 1 << (int(rows).bit_length() - 1)))


def _reduce_to(t, shape):
    """Sum ``t`` [B, H, rows, Sk] over the dims where ``shape`` (the bias, 4-D) broadcasts."""
    dims = [i for i in range(4) if shape[i] == 1 and t.shape[i] != 1]
    return t.sum(dim=dims, keepdim=True) if dims else t


class _ChunkedAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, bias, dropout_p, causal, scale, k_lens, block, seed):
        B, Sq, H, d = q.shape
        Sk = k.shape[1]
        qf = q.permute(0, 2, 1, 3)  # [B, H, Sq, d] views
        kf = k.permute(0, 2, 1, 3)
        vf = v.permute(0, 2, 1, 3)
        out = torch.empty(B, H, Sq, v.shape[-1], dtype=q.dtype, device=q.device)
        lse = torch.empty(B, H, Sq, dtype=torch.float32, device=q.device)
        kT = kf.float().transpose(-1, -2)
        vff = vf.float()
        keymask = None
        if k_lens is not None:
            keymask = torch.arange(Sk, device=q.device)[None, :] >= k_lens[:, None].long()  # [B, Sk]
        for i0 in range(0, Sq, block):
            i1 = min(Sq, i0 + block)
            s = _scores(qf, kT, bias, scale, causal, keymask, i0, i1)
            m = s.amax(-1, keepdim=True)
            m = torch.where(torch.isfinite(m), m, torch.zeros_like(m))
            p = torch.exp(s - m)
            l = p.sum(-1, keepdim=True)
            lse[:, :, i0:i1] = (m + torch.log(l)).squeeze(-1)
            p = p / l.clamp_min(1e-38) * (l > 0)
            if dropout_p > 0:
                p = p * _keep(p.shape, dropout_p, seed, i0, q.device)
            out[:, :, i0:i1] = torch.matmul(p, vff).to(q.dtype)
        ctx.save_for_backward(q, k, v, bias if bias is not None else torch.empty(0), out, lse,
                              k_lens if k_lens is not None else torch.empty(0))
        ctx.cfg = (dropout_p, causal, scale, block, seed, bias is not None, k_lens is not None)
        return out.permute(0, 2, 1, 3)

    @staticmethod
    def backward(ctx, do):
        q, k, v, bias, out, lse, k_lens = ctx.saved_tensors
        dropout_p, causal, scale, block, seed, has_bias, has_klens = ctx.cfg
        bias = bias if has_bias else None
        B, Sq, H, d = q.shape
        Sk = k.shape[1]
        qf = q.permute(0, 2, 1, 3).float()
        kf = k.permute(0, 2, 1, 3).float()
        vf = v.permute(0, 2, 1, 3).float()
        dof = do.permute(0, 2, 1, 3).float()
        kT = kf.transpose(-1, -2)
        keymask = None
        if has_klens:
            keymask = torch.arange(Sk, device=q.device)[None, :] >= k_lens[:, None].long()
        delta = (dof * out.float()).sum(-1)  # [B, H, Sq]
        dq = torch.empty_like(qf)
        dk = torch.zeros_like(kf)
        dv = torch.zeros_like(vf)
        need_db = has_bias and ctx.needs_input_grad[3]
        db = torch.zeros(bias.shape, dtype=torch.float32, device=q.device) if need_db else None
        for i0 in range(0, Sq, block):
            i1 = min(Sq, i0 + block)
            s = _scores(qf, kT, bias, scale, causal, keymask, i0, i1)
            p = torch.exp(s - lse[:, :, i0:i1, None])  # softmax probabilities (0 where masked)
            p = torch.nan_to_num(p, nan=0.0)
            dob = dof[:, :, i0:i1]
            if dropout_p > 0:
                keep = _keep(p.shape, dropout_p, seed, i0, q.device)
                pd = p * keep
                dp = torch.matmul(dob, vf.transpose(-1, -2)) * keep
            else:
                pd = p
                dp = torch.matmul(dob, vf.transpose(-1, -2))
            dv += torch.matmul(pd.transpose(-1, -2), dob)
            ds = p * (dp - delta[:, :, i0:i1, None])
            dq[:, :, i0:i1] = torch.matmul(ds, kf) * scale
            dk += torch.matmul(ds.transpose(-1, -2), qf[:, :, i0:i1]) * scale
            if need_db:
                part = _reduce_to(ds, db.shape)
                if db.shape[2] == 1:
                    db += part.sum(2, keepdim=True) if part.shape[2] != 1 else part
                else:
                    db[:, :, i0:i1] += part
        dq = dq.permute(0, 2, 1, 3).to(q.dtype)
        dk = dk.permute(0, 2, 1, 3).to(k.dtype)
        dv = dv.permute(0, 2, 1, 3).to(v.dtype)
        dbias = db.to(bias.dtype) if need_db else None
        return dq, dk, dv, dbias, None, None, None, None, None, None


def _scores(qf, kT, bias, scale, causal, keymask, i0, i1):
    s = torch.matmul(qf[:, :, i0:i1].float(), kT) * scale  # [B, H, rows, Sk] fp32
    if bias is not None:
        b = bias
        if b.dtype == torch.bool:
            b = torch.zeros(b.shape, device=b.device).masked_fill(~b, float("-inf"))
        b = b[:, :, i0:i1] if b.shape[2] != 1 else b
        s = s + b.float()
    if keymask is not None:
        s = s.masked_fill(keymask[:, None, None, :], float("-inf"))
    if causal:
        Sk = s.shape[-1]
        rows = torch.arange(i0, i1, device=s.device)[:, None]
        s = s.masked_fill(torch.arange(Sk, device=s.device)[None, :] > rows, float("-inf"))
    return s


def _keep(shape, p, seed, i0, device):
    g = torch.Generator(device=device)
    g.manual_seed(int(seed) * 1000003 + i0)
    return (torch.rand(shape, generator=g, device=device) >= p).float() / (1.0 - p)


def _bias4(bias, B, H, Sq, Sk):
    if bias is None:
        return None
    b = bias
    while b.dim() < 4:
        b = b.unsqueeze(0)
    if b.shape[-1] != Sk and b.shape[-1] == 1:
        b = b.expand(*b.shape[:-1], Sk)
    return b


def chunked_attention(q, k, v, attn_bias=None, dropout_p=0.0, causal=False, scale=None, k_lens=None,
                      block=None):
    """q: [B, Sq, h, d], k/v: [B, Sk, h, d] -> [B, Sq, h, d]; query-blocked, O(S * block) memory;
    ``attn_bias`` broadcastable to [B, h, Sq, Sk], may require a gradient."""
    B, Sq, H, d = q.shape
    Sk = k.shape[1]
    scale = 1.0 / math.sqrt(d) if scale is None else scale
    block = block or _block_rows(B, H, Sq, Sk)
    seed = 0
    if dropout_p > 0:
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,), device="cpu").item())
    bias = _bias4(attn_bias, B, H, Sq, Sk)
    return _ChunkedAttention.apply(q, k, v, bias, float(dropout_p), bool(causal), float(scale), k_lens, int(block),
                                   seed)
