"""apex.contrib.multihead_attn — fused self / encoder-decoder attention (NS-05)."""
from . import attention  # noqa: F401
