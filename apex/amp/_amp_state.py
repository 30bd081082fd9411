"""Process-global amp state (one per process; amp is configured once per job)."""
from __future__ import annotations


class AmpState:
    def __init__(self):
        self.hard_override = False
        self.allow_incoming_model_not_fp32 = False
        self.verbosity = 1
        self.opt_properties = None
        self.loss_scalers = []
        self.handle = None  # legacy amp.init() handle / new-API cast engine handle
        self.min_loss_scale = None
        self.max_loss_scale = 2.0 ** 24
        self.optimizers = []


_amp_state = AmpState()


def warn_or_err(msg):
    if _amp_state.hard_override:
        print("Warning:  " + msg)
    else:
        raise RuntimeError(msg)


def maybe_print(msg, rank0=False):
    import torch.distributed as dist

    if _amp_state.verbosity > 0:
        if rank0 and dist.is_available() and dist.is_initialized():
            if dist.get_rank() == 0:
                print(msg)
        else:
            print(msg)


def master_params(optimizer):
    """Generator over the (fp32 master) params an optimizer updates."""
    for group in optimizer.param_groups:
        for p in group["params"]:
            yield p
