"""GPT-2 (1.5B by default) — BASELINE.json config 4 ("GPT-2 1.5B with apex.contrib fused
multihead_attn + xentropy, DDP"). Written from scratch; random init, synthetic tokens.

Pre-LN decoder blocks; every hot op is an apex fused op on MI355X:
  LN (HIP FusedLayerNorm) -> fused QKV GEMM -> causal MFMA flash attention (apex.contrib)
  -> out-proj GEMM + bias/dropout/residual (one fused kernel each way)
  -> LN -> fc GEMM + bias/GELU(tanh) fused -> proj GEMM + bias/dropout/residual fused
  LM head tied to the token embedding, loss = apex.contrib.xentropy (fp32 statistics,
  never materialises fp32 logits). Vocab padded to a multiple of 64 (50257 -> 50304).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import torch
import torch.nn.functional as F
from torch import nn

from ..normalization import FusedLayerNorm
from ..ops import blocks as fblocks
from ..ops import fused as fops


# APEX_GPT_FUSED_LN=0: per-block forward (separate LayerNorms; A/B and fallback switch)
_FUSED_LN = os.environ.get("APEX_GPT_FUSED_LN", "1") != "0"

@dataclass
class GPTConfig:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 1600
    n_layer: int = 48
    n_head: int = 25
    dropout: float = 0.1
    layer_norm_eps: float = 1e-5
    initializer_range: float = 0.02
    pad_vocab_to: int = 64

    @property
    def padded_vocab(self):
        m = self.pad_vocab_to
        return (self.vocab_size + m - 1) // m * m

    @staticmethod
    def gpt2_1_5b():
        return GPTConfig()

    @staticmethod
    def gpt2_medium():
        return GPTConfig(n_embd=1024, n_layer=24, n_head=16)

    @staticmethod
    def tiny():
        return GPTConfig(vocab_size=1000, n_positions=128, n_embd=128, n_layer=2, n_head=2)


class GPTBlock(nn.Module):
    def __init__(self, c: GPTConfig):
        super().__init__()
        self.h, self.d = c.n_head, c.n_embd // c.n_head
        self.ln_1 = FusedLayerNorm(c.n_embd, eps=c.layer_norm_eps)
        self.c_attn = nn.Linear(c.n_embd, 3 * c.n_embd)
        self.c_proj = nn.Linear(c.n_embd, c.n_embd)
        self.ln_2 = FusedLayerNorm(c.n_embd, eps=c.layer_norm_eps)
        self.c_fc = nn.Linear(c.n_embd, 4 * c.n_embd)
        self.mlp_proj = nn.Linear(4 * c.n_embd, c.n_embd)
        self.p = c.dropout

    def forward(self, x):
        B, S, E = x.shape
        p = self.p if self.training else 0.0
        qkv = fops.fused_dense(self.ln_1(x), self.c_attn.weight, self.c_attn.bias).view(B, S, 3, self.h, self.d)
        ctx = fops.attention_qkv_packed(qkv, None, p, causal=True).reshape(B, S, E)
        x = fops.bias_dropout_add(fops.fused_dense(ctx, self.c_proj.weight, None), self.c_proj.bias, x, p)
        xn = self.ln_2(x)
        t = fblocks.mlp(xn, self.c_fc.weight, self.c_fc.bias, self.mlp_proj.weight, fops.ACT_GELU_TANH)
        if t is None:
            h = fops.dense_act(xn, self.c_fc.weight, self.c_fc.bias, fops.ACT_GELU_TANH)
            t = fops.fused_dense(h, self.mlp_proj.weight, None)
        return fops.bias_dropout_add(t, self.mlp_proj.bias, x, p)

    def forward_fused(self, x, xn, nxt):
        """The same block with its LayerNorms fused into the residual updates before them: takes the
        residual stream x and xn = ln_1(x), returns (x', nxt(x')) where nxt is the NEXT block's ln_1
        (or the final ln_f). Each residual update + the LayerNorm after it is one bdaln kernel each
        way (fops.bias_dropout_add_ln), so the stream is not re-read by a separate LayerNorm and its
        two gradients are summed inside the LayerNorm backward."""
        B, S, E = x.shape
        p = self.p if self.training else 0.0
        qkv = fops.fused_dense(xn, self.c_attn.weight, self.c_attn.bias).view(B, S, 3, self.h, self.d)
        ctx = fops.attention_qkv_packed(qkv, None, p, causal=True).reshape(B, S, E)
        x, xn = fops.bias_dropout_add_ln(fops.fused_dense(ctx, self.c_proj.weight, None), self.c_proj.bias, x,
                                         self.ln_2.weight, self.ln_2.bias, p, self.ln_2.eps)
        t = fblocks.mlp(xn, self.c_fc.weight, self.c_fc.bias, self.mlp_proj.weight, fops.ACT_GELU_TANH)
        if t is None:
            h = fops.dense_act(xn, self.c_fc.weight, self.c_fc.bias, fops.ACT_GELU_TANH)
            t = fops.fused_dense(h, self.mlp_proj.weight, None)
        return fops.bias_dropout_add_ln(t, self.mlp_proj.bias, x, nxt.weight, nxt.bias, p, nxt.eps)


class GPTModel(nn.Module):
    def __init__(self, c: GPTConfig):
        super().__init__()
        self.config = c
        self.wte = nn.Embedding(c.padded_vocab, c.n_embd)
        self.wpe = nn.Embedding(c.n_positions, c.n_embd)
        self.blocks = nn.ModuleList([GPTBlock(c) for _ in range(c.n_layer)])
        self.ln_f = FusedLayerNorm(c.n_embd, eps=c.layer_norm_eps)
        self.apply(self._init)
        for n, p in self.named_parameters():  # GPT-2 scaled init of residual projections
            if n.endswith("c_proj.weight") or n.endswith("mlp_proj.weight"):
                nn.init.normal_(p, 0.0, c.initializer_range / math.sqrt(2 * c.n_layer))

    def _init(self, m):
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, 0.0, self.config.initializer_range)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, 0.0, self.config.initializer_range)

    def forward(self, input_ids, labels=None):
        B, S = input_ids.shape
        if S > self.config.n_positions:  # host-side check: an out-of-range gather faults the GPU
            raise ValueError(f"sequence length {S} exceeds n_positions={self.config.n_positions}")
        pos = torch.arange(S, device=input_ids.device)
        x = self.wte(input_ids) + self.wpe(pos)[None]
        x = F.dropout(x, self.config.dropout, self.training)
        if len(self.blocks) and _FUSED_LN:
            # residual stream with each LayerNorm fused into the residual update before it
            xn = self.blocks[0].ln_1(x)
            for i, blk in enumerate(self.blocks):
                nxt = self.blocks[i + 1].ln_1 if i + 1 < len(self.blocks) else self.ln_f
                x, xn = blk.forward_fused(x, xn, nxt)
            x = xn
        else:
            for blk in self.blocks:
                x = blk(x)
            x = self.ln_f(x)
        logits = fops.fused_dense(x, self.wte.weight, None)
        if labels is None:
            return logits
        # shift the LABELS (not the [B, S, V] logits): the last position is ignored
        shifted = torch.cat([labels[:, 1:], torch.full_like(labels[:, :1], -1)], 1)
        return fops.softmax_cross_entropy(logits.view(-1, logits.shape[-1]), shifted.reshape(-1), ignore_index=-1)


def synthetic_batch(c: GPTConfig, batch, seq_len, device="cpu", generator=None):
    ids = torch.randint(0, c.vocab_size, (batch, seq_len), device=device, generator=generator)
    return dict(input_ids=ids, labels=ids)


def param_groups(model, weight_decay=0.01):
    decay, no_decay = [], []
    for n, p in model.named_parameters():
        (no_decay if p.ndim == 1 else decay).append(p)
    return [{"params": decay, "weight_decay": weight_decay}, {"params": no_decay, "weight_decay": 0.0}]
