"""BERT (Large by default) for pre-training — the headline workload of BASELINE.json
("BERT-Large pretrain amp O2 + FusedLAMB + FusedLayerNorm, DDP").

Written from scratch (no checkpoint / network access: random init, synthetic data).
Architecture: post-LN Transformer encoder, GELU FFN, MLM head tied to the word
embeddings evaluated only at the masked positions (max_predictions_per_seq), NSP head.

MI355X choices:
  * QKV projection is one [3H, H] GEMM (one hipBLASLt call instead of three);
  * LayerNorms are apex FusedLayerNorm (csrc/layer_norm.hip);
  * attention runs through apex.contrib.multihead_attn's fused attention core when the
    HIP kernels are present;
  * vocab padded to a multiple of 64 so the decoder GEMM N dimension tiles cleanly.
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


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 1024
    num_hidden_layers: int = 24
    num_attention_heads: int = 16
    intermediate_size: int = 4096
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    initializer_range: float = 0.02
    layer_norm_eps: float = 1e-12
    pad_vocab_to: int = 64

    @property
    def padded_vocab(self):
        m = self.pad_vocab_to
        return (self.vocab_size + m - 1) // m * m

    @staticmethod
    def large():
        return BertConfig()

    @staticmethod
    def base():
        return BertConfig(hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                          intermediate_size=3072)

    @staticmethod
    def tiny():
        return BertConfig(vocab_size=1000, hidden_size=128, num_hidden_layers=2,
                          num_attention_heads=2, intermediate_size=512, max_position_embeddings=128)


class BertEmbeddings(nn.Module):
    # one fused kernel each way (apex.ops.fused.bert_embeddings); APEX_BERT_EMBED_FUSION=0 selects
    # the op-by-op composition
    use_fused = os.environ.get("APEX_BERT_EMBED_FUSION", "1") == "1"

    def __init__(self, c: BertConfig):
        super().__init__()
        self.word_embeddings = nn.Embedding(c.padded_vocab, c.hidden_size)
        self.position_embeddings = nn.Embedding(c.max_position_embeddings, c.hidden_size)
        self.token_type_embeddings = nn.Embedding(c.type_vocab_size, c.hidden_size)
        self.LayerNorm = FusedLayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.p = c.hidden_dropout_prob

    def forward(self, input_ids, token_type_ids):
        S = input_ids.shape[1]
        if S > self.position_embeddings.num_embeddings:  # host-side check (a bad gather faults the GPU)
            raise ValueError(f"sequence length {S} exceeds max_position_embeddings="
                             f"{self.position_embeddings.num_embeddings}")
        if self.use_fused:
            return fops.bert_embeddings(input_ids, token_type_ids, self.word_embeddings.weight,
                                        self.position_embeddings.weight, self.token_type_embeddings.weight,
                                        self.LayerNorm.weight, self.LayerNorm.bias, self.p, self.LayerNorm.eps,
                                        training=self.training)
        pos = torch.arange(S, device=input_ids.device)
        x = self.word_embeddings(input_ids) + self.position_embeddings(pos)[None] + \
            self.token_type_embeddings(token_type_ids)
        x = self.LayerNorm(x)
        return F.dropout(x, self.p, self.training)


class BertSelfAttention(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.h = c.num_attention_heads
        self.d = c.hidden_size // c.num_attention_heads
        self.qkv = nn.Linear(c.hidden_size, 3 * c.hidden_size)
        self.dense = nn.Linear(c.hidden_size, c.hidden_size)
        self.p_attn = c.attention_probs_dropout_prob

    def context(self, x, k_lens):
        """Attention context [B, S, H] (before the output projection)."""
        B, S, H = x.shape
        qkv = fops.fused_dense(x, self.qkv.weight, self.qkv.bias).view(B, S, 3, self.h, self.d)
        ctx = fops.attention_qkv_packed(qkv, None, self.p_attn if self.training else 0.0, k_lens=k_lens)
        return ctx.reshape(B, S, H)

    def forward(self, x, k_lens):
        return fops.fused_dense(self.context(x, k_lens), self.dense.weight, self.dense.bias)


class BertLayer(nn.Module):
    """Post-LN encoder layer; each sublayer output is ONE fused kernel each way:
    LN(residual + dropout(x W^T + b)) (csrc/fused_ops.hip bdaln)."""

    def __init__(self, c: BertConfig):
        super().__init__()
        self.attention = BertSelfAttention(c)
        self.attn_ln = FusedLayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.intermediate = nn.Linear(c.hidden_size, c.intermediate_size)
        self.output = nn.Linear(c.intermediate_size, c.hidden_size)
        self.out_ln = FusedLayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.p = c.hidden_dropout_prob
        self.eps = c.layer_norm_eps

    # whole-sublayer Functions (apex/ops/blocks.py) on the MFMA GEMM with fused epilogues;
    # APEX_BERT_SUBLAYER_FUSION=0 selects the op-by-op composition (same numerics)
    use_sublayer_fusion = os.environ.get("APEX_BERT_SUBLAYER_FUSION", "1") == "1"

    def forward(self, x, k_lens):
        if self.use_sublayer_fusion:
            y = self._forward_sublayers(x, k_lens)
            if y is not None:
                return y
        p = self.p if self.training else 0.0
        ctx = self.attention.context(x, k_lens)
        d = self.attention.dense
        x = fops.dense_bias_dropout_add_ln(ctx, d.weight, d.bias, x, self.attn_ln.weight,
                                           self.attn_ln.bias, p, self.eps)
        h = fops.dense_gelu(x, self.intermediate.weight, self.intermediate.bias)
        return fops.dense_bias_dropout_add_ln(h, self.output.weight, self.output.bias, x,
                                              self.out_ln.weight, self.out_ln.bias, p, self.eps)

    def _forward_sublayers(self, x, k_lens):
        """Both sublayers as whole-sublayer Functions (apex/ops/blocks.py): the residual
        gradients ride in the input-gradient GEMMs' epilogues. None -> op-by-op path."""
        a = self.attention
        y = fblocks.attention_sublayer(x, a.qkv.weight, a.qkv.bias, a.dense.weight, a.dense.bias,
                                       self.attn_ln.weight, self.attn_ln.bias, a.h, a.p_attn, self.p,
                                       self.eps, k_lens=k_lens, training=self.training)
        if y is None:
            return None
        out = fblocks.ffn_sublayer(y, self.intermediate.weight, self.intermediate.bias, self.output.weight,
                                   self.output.bias, self.out_ln.weight, self.out_ln.bias, self.p, self.eps,
                                   training=self.training)
        if out is None:
            return fops.dense_bias_dropout_add_ln(
                fops.dense_gelu(y, self.intermediate.weight, self.intermediate.bias), self.output.weight,
                self.output.bias, y, self.out_ln.weight, self.out_ln.bias, self.p if self.training else 0.0,
                self.eps)
        return out


class BertModel(nn.Module):
    def __init__(self, c: BertConfig, add_pooling_layer=True):
        super().__init__()
        self.config = c
        self.embeddings = BertEmbeddings(c)
        self.layers = nn.ModuleList([BertLayer(c) for _ in range(c.num_hidden_layers)])
        self.pooler = nn.Linear(c.hidden_size, c.hidden_size) if add_pooling_layer else None

    def forward(self, input_ids, token_type_ids=None, attention_mask=None):
        if token_type_ids is None:
            token_type_ids = torch.zeros_like(input_ids)
        x = self.embeddings(input_ids, token_type_ids)
        # BERT batches are right-padded: the mask is a per-sequence valid length, which the
        # flash kernel consumes directly (no [B,1,1,S] additive bias tensor)
        k_lens = None
        if attention_mask is not None:
            k_lens = attention_mask.sum(1, dtype=torch.int32)
        for layer in self.layers:
            x = layer(x, k_lens)
        pooled = torch.tanh(self.pooler(x[:, 0])) if self.pooler is not None else None
        return x, pooled


class BertForPreTraining(nn.Module):
    """MLM (at ``masked_lm_positions``) + NSP heads; forward returns the total loss."""

    def __init__(self, c: BertConfig):
        super().__init__()
        self.config = c
        self.bert = BertModel(c)
        self.transform = nn.Linear(c.hidden_size, c.hidden_size)
        self.transform_ln = FusedLayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.decoder_bias = nn.Parameter(torch.zeros(c.padded_vocab))
        self.nsp = nn.Linear(c.hidden_size, 2)
        self.apply(self._init_weights)

    def _init_weights(self, m):
        std = self.config.initializer_range
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, 0.0, std)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, 0.0, std)

    def forward(self, input_ids, token_type_ids, attention_mask, masked_lm_positions,
                masked_lm_labels, next_sentence_labels):
        seq, pooled = self.bert(input_ids, token_type_ids, attention_mask)
        B, S, H = seq.shape
        P = masked_lm_positions.shape[1]
        idx = (masked_lm_positions + torch.arange(B, device=seq.device)[:, None] * S).reshape(-1)
        sel = seq.reshape(B * S, H).index_select(0, idx)
        t = fops.linear_gelu(sel, self.transform.weight, self.transform.bias)
        t = self.transform_ln(t)
        logits = fops.fused_dense(t, self.bert.embeddings.word_embeddings.weight, self.decoder_bias)
        labels = masked_lm_labels.reshape(-1)
        mlm = fops.softmax_cross_entropy(logits, labels, ignore_index=-1)
        nsp = fops.softmax_cross_entropy(self.nsp(pooled), next_sentence_labels, ignore_index=-1)
        return mlm + nsp


def synthetic_batch(c: BertConfig, batch, seq_len, max_pred=None, device="cpu", generator=None):
    """Synthetic pre-training batch of the exact shapes the real pipeline produces."""
    max_pred = max_pred or max(1, int(round(seq_len * 0.15)))
    g = generator
    input_ids = torch.randint(0, c.vocab_size, (batch, seq_len), device=device, generator=g)
    token_type = torch.zeros(batch, seq_len, dtype=torch.long, device=device)
    token_type[:, seq_len // 2:] = 1
    attn = torch.ones(batch, seq_len, dtype=torch.long, device=device)
    pos = torch.stack([torch.randperm(seq_len - 1, device=device, generator=g)[:max_pred] + 1
                       for _ in range(batch)]).sort(dim=1).values
    labels = torch.randint(0, c.vocab_size, (batch, max_pred), device=device, generator=g)
    nsp = torch.randint(0, 2, (batch,), device=device, generator=g)
    return dict(input_ids=input_ids, token_type_ids=token_type, attention_mask=attn,
                masked_lm_positions=pos, masked_lm_labels=labels, next_sentence_labels=nsp)


def param_groups_for_lamb(model, weight_decay=0.01):
    """Standard BERT grouping: no weight decay on biases and LayerNorm params."""
    decay, no_decay = [], []
    for n, p in model.named_parameters():
        if not p.requires_grad:
            continue
        if p.ndim == 1 or n.endswith(".bias") or "LayerNorm" in n or "_ln" in n:
            no_decay.append(p)
        else:
            decay.append(p)
    return [{"params": decay, "weight_decay": weight_decay},
            {"params": no_decay, "weight_decay": 0.0}]
