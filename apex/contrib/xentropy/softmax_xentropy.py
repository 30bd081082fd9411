"""Softmax cross-entropy autograd function over csrc/xentropy.hip."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ... import _ext


def _reference_rows(logits, labels, smoothing, padding_idx):
    lf = logits.float()
    lse = torch.logsumexp(lf, dim=-1)
    valid = labels != padding_idx
    safe = labels.clamp(0, lf.shape[-1] - 1)
    xy = lf.gather(-1, safe[:, None]).squeeze(-1)
    loss = (1 - smoothing) * (lse - xy) + smoothing * (lse - lf.mean(-1))
    return torch.where(valid, loss, torch.zeros_like(loss))


class SoftmaxCrossEntropyLoss(torch.autograd.Function):
    """Per-row fp32 losses; rows labelled ``padding_idx`` contribute 0 loss / 0 grad."""

    @staticmethod
    def forward(ctx, logits, labels, smoothing=0.0, padding_idx=0, half_to_float=False):
        C = _ext.require()
        lg = logits.contiguous()
        losses, lse = C.xent_fwd(lg, labels, float(smoothing), int(padding_idx))
        ctx.save_for_backward(lg, lse, labels)
        ctx.smoothing, ctx.padding_idx = smoothing, padding_idx
        return losses

    @staticmethod
    def backward(ctx, grad_loss):
        C = _ext.require()
        lg, lse, labels = ctx.saved_tensors
        g = grad_loss if grad_loss.dtype == torch.float32 else grad_loss.float()
        dx = C.xent_bwd(g, lg, lse, labels, float(ctx.smoothing), int(ctx.padding_idx))
        return dx, None, None, None, None


def softmax_xentropy(logits, labels, smoothing=0.0, ignore_index=-100, reduction="mean"):
    """Functional form: ``reduction`` in {'none', 'sum', 'mean'}; mean is over the
    non-ignored rows and is computed on the device (no host sync)."""
    if logits.dim() != 2:
        logits = logits.reshape(-1, logits.shape[-1])
        labels = labels.reshape(-1)
    if _ext.use_native(logits):
        rows = SoftmaxCrossEntropyLoss.apply(logits, labels, smoothing, ignore_index, False)
    else:
        if smoothing == 0.0:
            rows = F.cross_entropy(logits.float(), labels, ignore_index=ignore_index, reduction="none")
        else:
            rows = _reference_rows(logits, labels, smoothing, ignore_index)
    if reduction == "none":
        return rows
    if reduction == "sum":
        return rows.sum()
    count = (labels != ignore_index).sum().clamp(min=1)
    return rows.sum() / count
