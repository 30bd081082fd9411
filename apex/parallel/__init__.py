"""apex.parallel — data parallelism over RCCL/xGMI for MI355X (R-15..R-19, NS-04).

Reference exports (apex/parallel/__init__.py:1): DistributedDataParallel, Reducer.
LARC is exported here too (the reference forgot to).
"""
from .distributed import DistributedDataParallel, Reducer, flat_dist_call, apply_flat_dist_call, grad_target
from .LARC import LARC

try:
    from .sync_batchnorm import SyncBatchNorm, convert_syncbn_model, create_syncbn_process_group
except ImportError:  # pragma: no cover - during bring-up
    pass

__all__ = ["DistributedDataParallel", "Reducer", "LARC", "SyncBatchNorm", "convert_syncbn_model",
           "create_syncbn_process_group", "flat_dist_call", "apply_flat_dist_call", "grad_target"]
