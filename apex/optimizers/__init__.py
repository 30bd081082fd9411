"""apex.optimizers — HIP-fused optimizers for MI355X (NS-02)."""
from .fused_adam import FusedAdam
from .fused_lamb import FusedLAMB
from .fused_sgd import FusedSGD

__all__ = ["FusedAdam", "FusedLAMB", "FusedSGD"]
