"""Vocab-parallel softmax cross-entropy (NS-08): logits stay sharded over the TP group.

Forward: local max -> all-reduce(MAX); local sum-exp -> all-reduce(SUM); the target logit
is picked by the rank that owns it and all-reduced (SUM). Only three [tokens]-sized
collectives per step, never the [tokens, vocab] logits. Label smoothing supported.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ... import _ext
from .. import parallel_state as ps
from .utils import VocabUtility


class _VocabParallelCrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, vocab_parallel_logits, target, label_smoothing=0.0):
        group = ps.get_tensor_model_parallel_group()
        logits = vocab_parallel_logits.float()
        logits_max = logits.max(dim=-1)[0]
        dist.all_reduce(logits_max, op=dist.ReduceOp.MAX, group=group)
        logits = logits - logits_max.unsqueeze(-1)
        part = logits.shape[-1]
        rank, ws = ps.get_tensor_model_parallel_rank(), ps.get_tensor_model_parallel_world_size()
        start, end = VocabUtility.vocab_range_from_per_partition_vocab_size(part, rank, ws)
        target_mask = (target < start) | (target >= end)
        masked_target = (target - start).clamp(0, part - 1)
        masked_target = masked_target.masked_fill(target_mask, 0)
        l2d = logits.view(-1, part)
        pred = l2d.gather(1, masked_target.view(-1, 1)).view(target.shape)
        pred = pred.masked_fill(target_mask, 0.0)
        dist.all_reduce(pred, group=group)
        exp_logits = logits.exp()
        sum_exp = exp_logits.sum(dim=-1)
        dist.all_reduce(sum_exp, group=group)
        loss = torch.log(sum_exp) - pred
        vocab_size = part * ws
        if label_smoothing > 0:
            smoothing = label_smoothing * vocab_size / (vocab_size - 1)
            log_probs = logits - torch.log(sum_exp).unsqueeze(-1)
            mean_log = log_probs.sum(-1)
            dist.all_reduce(mean_log, group=group)
            mean_log = mean_log / vocab_size
            loss = (1.0 - smoothing) * loss - smoothing * mean_log
        else:
            smoothing = 0.0
        exp_logits.div_(sum_exp.unsqueeze(-1))
        ctx.save_for_backward(exp_logits, target_mask, masked_target)
        ctx.cfg = (smoothing, vocab_size)
        return loss

    @staticmethod
    def backward(ctx, grad_output):
        softmax, target_mask, masked_target = ctx.saved_tensors
        smoothing, vocab_size = ctx.cfg
        grad = softmax
        part = softmax.shape[-1]
        g2d = grad.view(-1, part)
        rows = torch.arange(g2d.shape[0], device=g2d.device)
        upd = 1.0 - target_mask.view(-1).float()
        if smoothing > 0:
            g2d[rows, masked_target.view(-1)] -= (1.0 - smoothing) * upd
            g2d -= smoothing / vocab_size
        else:
            g2d[rows, masked_target.view(-1)] -= upd
        grad.mul_(grad_output.unsqueeze(-1))
        return grad, None, None


def vocab_parallel_cross_entropy(vocab_parallel_logits, target, label_smoothing=0.0):
    """Per-token losses, shape of ``target``. At TP = 1 on the device the whole vocabulary is local:
    the fused HIP softmax cross-entropy (csrc/xentropy.hip) runs on the 16-bit logits directly —
    one pass each way, fp32 statistics, no fp32 copy of the [tokens, vocab] logits and no saved
    softmax (the torch composition below keeps both: 2 x 1.6 GB at Megatron's 8192 x 50304)."""
    lg = vocab_parallel_logits
    if (ps.get_tensor_model_parallel_world_size() == 1 and lg.dtype in (torch.float16, torch.bfloat16)
            and _ext.use_native(lg)):
        from ...contrib.xentropy import SoftmaxCrossEntropyLoss

        V = lg.shape[-1]
        # Megatron's smoothing convention: s' = s V / (V - 1) over (1 - s') (lse - x_y) + s' (lse - mean x)
        sm = float(label_smoothing) * V / (V - 1) if label_smoothing > 0 else 0.0
        rows = SoftmaxCrossEntropyLoss.apply(lg.reshape(-1, V), target.reshape(-1), sm, -100, False)
        return rows.view(target.shape)
    return _VocabParallelCrossEntropy.apply(vocab_parallel_logits, target, label_smoothing)
