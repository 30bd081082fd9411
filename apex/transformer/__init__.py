"""apex.transformer — Megatron-style tensor / pipeline / sequence / context parallelism for MI355X
(NS-08).

Process groups (parallel_state), TP layers and mappings (tensor_parallel), pipeline
schedules (pipeline_parallel), ring / Ulysses attention over a sharded sequence
(context_parallel), fused scale-mask softmax (functional), microbatch calculators. All
communication is RCCL through torch.distributed.
"""
from . import enums, parallel_state, tensor_parallel  # noqa: F401
from . import pipeline_parallel  # noqa: F401
from . import functional  # noqa: F401
from . import context_parallel  # noqa: F401
from .enums import AttnMaskType, AttnType, LayerType, ModelType  # noqa: F401
