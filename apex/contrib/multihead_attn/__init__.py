"""apex.contrib.multihead_attn — fused self / encoder-decoder attention (NS-05)."""
from . import attention  # noqa: F401
from .modules import EncdecMultiheadAttn, SelfMultiheadAttn

__all__ = ["SelfMultiheadAttn", "EncdecMultiheadAttn"]
