"""apex.ops — functional fused ops (HIP kernels with PyTorch reference formulations)."""
from . import fused  # noqa: F401
