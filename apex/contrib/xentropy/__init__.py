"""apex.contrib.xentropy — fused softmax cross-entropy with label smoothing (NS-06).

``SoftmaxCrossEntropyLoss.apply(logits, labels, smoothing=0.0, padding_idx=0,
half_to_float=False)`` follows apex's contrib API: per-row losses (fp32), rows whose
label equals ``padding_idx`` get zero loss and zero grad.
"""
from .softmax_xentropy import SoftmaxCrossEntropyLoss, softmax_xentropy

__all__ = ["SoftmaxCrossEntropyLoss", "softmax_xentropy"]
