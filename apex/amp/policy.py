"""amp cast-policy tables (R-08): what runs in low precision, what in fp32, what promotes.

Spec source: apex/amp/lists/functional_overrides.py:18-73, torch_overrides.py:5-93,
tensor_overrides.py:14-63. Held here as one table keyed by namespace
so the engine (wrap.py) can apply them uniformly; ``apex.amp.lists.*`` re-export the
per-namespace views for API compatibility.

Categories:
  low       -> cast fp32 inputs to the low-precision dtype (GEMM / conv class)
  fp32      -> cast low-precision inputs to fp32 (reductions, transcendental, losses)
  promote   -> if inputs mix low precision and fp32, run in fp32
  sequence  -> promote across a sequence argument (cat / stack)
  banned    -> error on low-precision inputs (or fp32 with allow_banned)
"""
from __future__ import annotations

import torch
import torch.nn.functional

_CONV = ["conv1d", "conv2d", "conv3d", "conv_transpose1d", "conv_transpose2d",
         "conv_transpose3d", "conv_tbc"]

_BCE_MSG = (
    "\namp does not work out-of-the-box with `F.binary_cross_entropy` or `torch.nn.BCELoss.` "
    "It requires that the output of the previous function be already a FloatTensor. \n\n"
    "Most models have a Sigmoid right before BCELoss. In that case, you can use\n"
    "    torch.nn.BCEWithLogitsLoss\nto combine Sigmoid+BCELoss into a single layer "
    "that is compatible with amp.\nAnother option is to add\n"
    "    amp.register_float_function(torch, 'sigmoid')\nbefore calling `amp.init()`.\n"
    "If you _really_ know what you are doing, you can disable this warning by passing "
    "allow_banned=True to `amp.init()`.")

FUNCTIONAL = {
    "module": torch.nn.functional,
    "low": _CONV + ["linear"],
    "fp32": [
        # pointwise
        "softplus", "softmin", "log_softmax", "softmax",
        # normalisation
        "layer_norm", "group_norm", "local_response_norm", "normalize", "cosine_similarity",
        # losses
        "poisson_nll_loss", "cosine_embedding_loss", "cross_entropy", "hinge_embedding_loss",
        "kl_div", "l1_loss", "mse_loss", "margin_ranking_loss", "multilabel_margin_loss",
        "multilabel_soft_margin_loss", "multi_margin_loss", "nll_loss",
        "binary_cross_entropy_with_logits", "smooth_l1_loss", "soft_margin_loss",
        "triplet_margin_loss",
    ],
    "promote": [],
    "sequence": [],
    "banned": [("binary_cross_entropy", _BCE_MSG)],
}

TORCH = {
    "module": torch,
    "low": _CONV + ["addmm", "addmv", "addr", "matmul", "mm", "mv"],
    "fp32": [
        # pointwise
        "acos", "asin", "cosh", "erfinv", "exp", "expm1", "log", "log10", "log2", "reciprocal",
        "rsqrt", "sinh", "tan", "pow",
        # reductions
        "cumprod", "cumsum", "dist", "mean", "norm", "prod", "std", "sum", "var",
        # reduction-like BLAS (bmm is fp32 in the reference policy)
        "addbmm", "baddbmm", "bmm",
        "renorm",
    ],
    "promote": ["addcdiv", "addcmul", "atan2", "cross", "add", "div", "mul",
                "eq", "equal", "ge", "gt", "le", "lt", "ne"],
    "sequence": ["cat", "stack"],
    "banned": [],
}

_TENSOR_OWN = {
    "low": ["__matmul__"],
    "fp32": ["__ipow__", "__pow__", "__rpow__", "cpu"],
    "promote": ["__add__", "__div__", "__eq__", "__ge__", "__gt__", "__iadd__", "__idiv__",
                "__imul__", "__isub__", "__itruediv__", "__le__", "__lt__", "__mul__", "__ne__",
                "__radd__", "__rdiv__", "__rmul__", "__rsub__", "__rtruediv__", "__sub__",
                "__truediv__"],
    "sequence": [],
}


def _tensor_table():
    t = {"module": torch.Tensor, "banned": []}
    for cat, names in _TENSOR_OWN.items():
        merged = list(names)
        # every torch-namespace entry that also exists as a Tensor method (tensor_overrides.py:58-63)
        for fn in TORCH[cat]:
            if hasattr(torch.Tensor, fn) and fn not in merged:
                merged.append(fn)
        t[cat] = merged
    return t


TENSOR = _tensor_table()

TABLES = (FUNCTIONAL, TORCH, TENSOR)

# RNN entry points (torch.nn.modules.rnn._VF) run in low precision (rnn_compat.py)
RNN_NAMES = ["rnn_relu", "rnn_tanh", "gru", "lstm"]
