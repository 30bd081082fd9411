"""apex.transformer.pipeline_parallel — 1F1B pipeline schedules over RCCL p2p (NS-08)."""
from . import p2p_communication  # noqa: F401
from .schedules import (forward_backward_no_pipelining, forward_backward_pipelining_without_interleaving,
                        get_forward_backward_func)
from .utils import (average_losses_across_data_parallel_group, get_num_microbatches,
                    setup_microbatch_calculator, update_num_microbatches)
