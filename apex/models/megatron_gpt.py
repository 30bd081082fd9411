"""Megatron-style GPT over apex.transformer — BASELINE.json config 5 ("apex.transformer
Megatron-style GPT, TP=4 PP=2 over xGMI on 8x MI355X").

Each pipeline stage owns a contiguous range of decoder layers; layer internals are
tensor-parallel: QKV and fc1 are ColumnParallelLinear (heads / FFN columns split across the
TP group, no gather), out-proj and fc2 are RowParallelLinear (one RCCL all-reduce each),
attention runs the causal MFMA flash kernel on the rank-local heads. Stage 0 holds the
vocab-parallel token embedding, the last stage the vocab-parallel LM head (tied to the
embedding: its gradient is all-reduced over the embedding group) and computes
vocab_parallel_cross_entropy on sharded logits.
"""
from __future__ import annotations

import contextlib
import math
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import nn

from ..normalization import FusedLayerNorm
from ..ops import blocks as fblocks
from ..ops import fused as fops
from ..transformer import parallel_state as ps
from ..transformer import tensor_parallel as tp


# APEX_MEGATRON_FUSED_LN=0: per-layer forward (separate LayerNorms; A/B and fallback switch)
_FUSED_LN = os.environ.get("APEX_MEGATRON_FUSED_LN", "1") != "0"

@dataclass
class MegatronGPTConfig:
    vocab_size: int = 50304
    hidden_size: int = 2048
    num_layers: int = 24
    num_attention_heads: int = 16
    ffn_hidden_size: int = None
    max_position_embeddings: int = 2048
    hidden_dropout: float = 0.1
    attention_dropout: float = 0.1
    layernorm_epsilon: float = 1e-5
    init_method_std: float = 0.02
    params_dtype: torch.dtype = torch.float32

    def __post_init__(self):
        if self.ffn_hidden_size is None:
            self.ffn_hidden_size = 4 * self.hidden_size

    @staticmethod
    def tiny():
        return MegatronGPTConfig(vocab_size=512, hidden_size=128, num_layers=4, num_attention_heads=4,
                                 max_position_embeddings=64)


def _init(std):
    return lambda w: nn.init.normal_(w, 0.0, std)


def _tp_rng():
    """Dropout on tensor-parallel shards (attention probabilities) draws from the tracked
    'model-parallel-rng' state: a different mask on every TP rank, the same on DP replicas."""
    tr = tp.get_cuda_rng_tracker()
    return tr.fork() if "model-parallel-rng" in tr.get_states() else contextlib.nullcontext()


class ParallelTransformerLayer(nn.Module):
    def __init__(self, c: MegatronGPTConfig, layer_number):
        super().__init__()
        tpws = ps.get_tensor_model_parallel_world_size()
        self.heads_local = tp.divide(c.num_attention_heads, tpws)
        self.d = c.hidden_size // c.num_attention_heads
        out_std = c.init_method_std / math.sqrt(2.0 * c.num_layers)
        self.input_layernorm = FusedLayerNorm(c.hidden_size, eps=c.layernorm_epsilon)
        self.query_key_value = tp.ColumnParallelLinear(c.hidden_size, 3 * c.hidden_size, gather_output=False,
                                                       init_method=_init(c.init_method_std),
                                                       params_dtype=c.params_dtype)
        self.dense = tp.RowParallelLinear(c.hidden_size, c.hidden_size, input_is_parallel=True,
                                          init_method=_init(out_std), skip_bias_add=True, params_dtype=c.params_dtype)
        self.post_attention_layernorm = FusedLayerNorm(c.hidden_size, eps=c.layernorm_epsilon)
        self.dense_h_to_4h = tp.ColumnParallelLinear(c.hidden_size, c.ffn_hidden_size, gather_output=False,
                                                     init_method=_init(c.init_method_std), skip_bias_add=True,
                                                     params_dtype=c.params_dtype)
        self.dense_4h_to_h = tp.RowParallelLinear(c.ffn_hidden_size, c.hidden_size, input_is_parallel=True,
                                                  init_method=_init(out_std), skip_bias_add=True,
                                                  params_dtype=c.params_dtype)
        self.p_hidden, self.p_attn = c.hidden_dropout, c.attention_dropout

    def forward(self, x):
        B, S, _ = x.shape
        ph = self.p_hidden if self.training else 0.0
        pa = self.p_attn if self.training else 0.0
        qkv, _ = self.query_key_value(self.input_layernorm(x))
        qkv = qkv.view(B, S, 3, self.heads_local, self.d)
        with _tp_rng():
            ctx = fops.attention_qkv_packed(qkv, None, pa, causal=True)
        out, bias = self.dense(ctx.reshape(B, S, -1))
        x = fops.bias_dropout_add(out, bias, x, ph)
        xn = self.post_attention_layernorm(x)
        f1, f2 = self.dense_h_to_4h, self.dense_4h_to_h
        if not (f1.sequence_parallel_enabled or f2.sequence_parallel_enabled) and f1.bias is not None:
            # whole MLP shard as one Function (GEMM+bias+GELU epilogue, dGELU epilogue in backward)
            # between the same TP mappings the two parallel linears apply
            t = fblocks.mlp(tp.copy_to_tensor_model_parallel_region(xn), f1.weight, f1.bias, f2.weight)
            if t is not None:
                return fops.bias_dropout_add(tp.reduce_from_tensor_model_parallel_region(t), f2.bias, x, ph)
        h, b1 = f1(xn)
        h = fops.bias_gelu(h, b1) if b1 is not None else F.gelu(h)
        out, bias = f2(h)
        return fops.bias_dropout_add(out, bias, x, ph)

    def forward_fused(self, x, xn, nxt):
        """forward() with each residual update fused with the LayerNorm after it (one bdaln kernel
        each way, fops.bias_dropout_add_ln): takes x and xn = input_layernorm(x), returns
        (x', nxt(x')) with nxt the next layer's input_layernorm / the final LayerNorm, or (x', None)
        at a pipeline-stage boundary (the next stage normalises its own input)."""
        B, S, _ = x.shape
        ph = self.p_hidden if self.training else 0.0
        pa = self.p_attn if self.training else 0.0
        qkv, _ = self.query_key_value(xn)
        qkv = qkv.view(B, S, 3, self.heads_local, self.d)
        with _tp_rng():
            ctx = fops.attention_qkv_packed(qkv, None, pa, causal=True)
        out, bias = self.dense(ctx.reshape(B, S, -1))
        ln2 = self.post_attention_layernorm
        x, xn = fops.bias_dropout_add_ln(out, bias, x, ln2.weight, ln2.bias, ph, ln2.eps)
        f1, f2 = self.dense_h_to_4h, self.dense_4h_to_h
        t = bias2 = None
        if not (f1.sequence_parallel_enabled or f2.sequence_parallel_enabled) and f1.bias is not None:
            t = fblocks.mlp(tp.copy_to_tensor_model_parallel_region(xn), f1.weight, f1.bias, f2.weight)
            if t is not None:
                t, bias2 = tp.reduce_from_tensor_model_parallel_region(t), f2.bias
        if t is None:
            h, b1 = f1(xn)
            h = fops.bias_gelu(h, b1) if b1 is not None else F.gelu(h)
            t, bias2 = f2(h)
        if nxt is None:
            return fops.bias_dropout_add(t, bias2, x, ph), None
        return fops.bias_dropout_add_ln(t, bias2, x, nxt.weight, nxt.bias, ph, nxt.eps)


class MegatronGPT(nn.Module):
    """One pipeline stage of the GPT (pre_process: embeddings, post_process: head + loss)."""

    def __init__(self, c: MegatronGPTConfig, pre_process=True, post_process=True, layer_offset=0,
                 num_local_layers=None):
        super().__init__()
        self.config = c
        self.pre_process, self.post_process = pre_process, post_process
        n = c.num_layers if num_local_layers is None else num_local_layers
        if pre_process:
            self.word_embeddings = tp.VocabParallelEmbedding(c.vocab_size, c.hidden_size,
                                                             init_method=_init(c.init_method_std),
                                                             params_dtype=c.params_dtype)
            self.position_embeddings = nn.Embedding(c.max_position_embeddings, c.hidden_size)
            nn.init.normal_(self.position_embeddings.weight, 0.0, c.init_method_std)
        self.layers = nn.ModuleList([ParallelTransformerLayer(c, layer_offset + i + 1) for i in range(n)])
        if post_process:
            self.final_layernorm = FusedLayerNorm(c.hidden_size, eps=c.layernorm_epsilon)
            if not pre_process:
                # LM head copy of the (tied) embedding on the last stage; grads synced over the
                # embedding group (first + last stage)
                self.word_embeddings = tp.VocabParallelEmbedding(c.vocab_size, c.hidden_size,
                                                                 init_method=_init(c.init_method_std),
                                                                 params_dtype=c.params_dtype)
        self.input_tensor = None

    def set_input_tensor(self, input_tensor):
        self.input_tensor = input_tensor

    def forward(self, input_ids, labels=None):
        if self.pre_process:
            S = input_ids.shape[1]
            if S > self.config.max_position_embeddings:  # host-side check (a bad gather faults the GPU)
                raise ValueError(f"sequence length {S} exceeds max_position_embeddings="
                                 f"{self.config.max_position_embeddings}")
            pos = torch.arange(S, device=input_ids.device)
            x = self.word_embeddings(input_ids) + self.position_embeddings(pos)[None]
            x = F.dropout(x, self.config.hidden_dropout, self.training)
        else:
            x = self.input_tensor
        if _FUSED_LN and len(self.layers):
            # residual stream with each LayerNorm fused into the residual update before it
            xn = self.layers[0].input_layernorm(x)
            for i, layer in enumerate(self.layers):
                if i + 1 < len(self.layers):
                    nxt = self.layers[i + 1].input_layernorm
                else:
                    nxt = self.final_layernorm if self.post_process else None
                x, xn = layer.forward_fused(x, xn, nxt)
            if self.post_process:
                return self._head(xn, labels)
            return x
        for layer in self.layers:
            x = layer(x)
        if not self.post_process:
            return x
        return self._head(self.final_layernorm(x), labels)

    def _head(self, x, labels):
        logits = fops.fused_dense(tp.copy_to_tensor_model_parallel_region(x), self.word_embeddings.weight, None)
        if labels is None:
            return logits
        shifted = torch.cat([labels[:, 1:], labels[:, -1:]], 1)
        loss = tp.vocab_parallel_cross_entropy(logits, shifted)  # fp32 statistics inside
        return loss[:, :-1].mean()


def build_stage(c: MegatronGPTConfig):
    """The GPT stage for this rank's pipeline position (layers split evenly)."""
    pp = ps.get_pipeline_model_parallel_world_size()
    r = ps.get_pipeline_model_parallel_rank()
    per = tp.divide(c.num_layers, pp)
    return MegatronGPT(c, pre_process=(r == 0), post_process=(r == pp - 1), layer_offset=r * per,
                       num_local_layers=per)


def sync_embedding_grads(model):
    """All-reduce the tied word-embedding grad between the first and last pipeline stage."""
    if ps.get_pipeline_model_parallel_world_size() == 1 or not ps.is_rank_in_embedding_group(True):
        return
    if not (model.pre_process or model.post_process):
        return
    w = model.word_embeddings.weight
    g = getattr(w, "main_grad", None)  # apex DDP fp32_main_grad mode: the fp32 accumulator
    if g is None:
        g = w.grad
        if g is None:
            g = torch.zeros_like(w)
            w.grad = g
    dist.all_reduce(g, group=ps.get_embedding_group())


def sync_initial_embeddings(model):
    """Make the last stage's LM-head copy equal to stage 0's embedding (call once)."""
    if ps.get_pipeline_model_parallel_world_size() == 1 or not ps.is_rank_in_embedding_group(True):
        return
    if not (model.pre_process or model.post_process):
        return
    w = model.word_embeddings.weight
    with torch.no_grad():
        if not model.pre_process:
            w.zero_()
        dist.all_reduce(w.data, group=ps.get_embedding_group())
