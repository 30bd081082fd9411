"""apex.transformer.tensor_parallel — Megatron-style tensor parallelism over RCCL (NS-08)."""
from .cross_entropy import vocab_parallel_cross_entropy
from .data import broadcast_data
from .layers import (ColumnParallelLinear, RowParallelLinear, VocabParallelEmbedding,
                     copy_tensor_model_parallel_attributes, param_is_not_tensor_parallel_duplicate,
                     set_defaults_if_not_set_tensor_model_parallel_attributes,
                     set_tensor_model_parallel_attributes)
from .mappings import (copy_to_tensor_model_parallel_region, gather_from_sequence_parallel_region,
                       gather_from_tensor_model_parallel_region, reduce_from_tensor_model_parallel_region,
                       reduce_scatter_to_sequence_parallel_region, scatter_to_sequence_parallel_region,
                       scatter_to_tensor_model_parallel_region)
from .random import checkpoint, get_cuda_rng_tracker, model_parallel_cuda_manual_seed
from .utils import VocabUtility, divide, split_tensor_along_last_dim
