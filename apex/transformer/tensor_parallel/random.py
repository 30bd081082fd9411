"""TP-aware RNG state tracking and activation checkpointing (NS-08).

Dropout inside tensor-parallel regions must differ across TP ranks (each holds a
different shard) but agree across DP replicas; ``model_parallel_cuda_manual_seed`` sets
the default generator to ``seed`` and a tracked "model-parallel-rng" state to
``seed + 2718 + tp_rank``. ``CheckpointFunction`` recomputes a block in backward with the
RNG states it saw in forward.
"""
from __future__ import annotations

import contextlib

import torch
from torch.utils.checkpoint import detach_variable

from .. import parallel_state as ps

_MODEL_PARALLEL_RNG_TRACKER_NAME = "model-parallel-rng"


def _dev_get_state():
    return torch.cuda.get_rng_state() if torch.cuda.is_available() else torch.get_rng_state()


def _dev_set_state(state):
    if torch.cuda.is_available():
        torch.cuda.set_rng_state(state)
    else:
        torch.set_rng_state(state)


class CudaRNGStatesTracker:
    def __init__(self):
        self.states_ = {}
        self.seeds_ = set()

    def reset(self):
        self.states_ = {}
        self.seeds_ = set()

    def get_states(self):
        return dict(self.states_)

    def set_states(self, states):
        self.states_ = states

    def add(self, name, seed):
        if seed in self.seeds_:
            raise Exception("seed {} already exists".format(seed))
        self.seeds_.add(seed)
        if name in self.states_:
            raise Exception("cuda rng state {} already exists".format(name))
        orig = _dev_get_state()
        if torch.cuda.is_available():
            torch.cuda.manual_seed(seed)
        else:
            torch.manual_seed(seed)
        self.states_[name] = _dev_get_state()
        _dev_set_state(orig)

    @contextlib.contextmanager
    def fork(self, name=_MODEL_PARALLEL_RNG_TRACKER_NAME):
        if name not in self.states_:
            raise Exception("cuda rng state {} is not added".format(name))
        orig = _dev_get_state()
        _dev_set_state(self.states_[name])
        try:
            yield
        finally:
            self.states_[name] = _dev_get_state()
            _dev_set_state(orig)


_CUDA_RNG_STATE_TRACKER = CudaRNGStatesTracker()


def get_cuda_rng_tracker():
    return _CUDA_RNG_STATE_TRACKER


def model_parallel_cuda_manual_seed(seed):
    offset = seed + 2718
    tp_seed = offset + ps.get_tensor_model_parallel_rank()
    data_parallel_seed = seed
    _CUDA_RNG_STATE_TRACKER.reset()
    if torch.cuda.is_available():
        torch.cuda.manual_seed(data_parallel_seed)
    torch.manual_seed(data_parallel_seed)
    _CUDA_RNG_STATE_TRACKER.add(_MODEL_PARALLEL_RNG_TRACKER_NAME, tp_seed)


class CheckpointFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, run_function, distribute_saved_activations, *args):
        ctx.run_function = run_function
        ctx.fwd_cpu_rng_state = torch.get_rng_state()
        ctx.fwd_dev_rng_state = _dev_get_state()
        ctx.fwd_tracker_states = get_cuda_rng_tracker().get_states()
        with torch.no_grad():
            outputs = run_function(*args)
        ctx.save_for_backward(*args)
        return outputs

    @staticmethod
    def backward(ctx, *grads):
        inputs = ctx.saved_tensors
        cpu_state, dev_state = torch.get_rng_state(), _dev_get_state()
        tracker = get_cuda_rng_tracker().get_states()
        torch.set_rng_state(ctx.fwd_cpu_rng_state)
        _dev_set_state(ctx.fwd_dev_rng_state)
        get_cuda_rng_tracker().set_states(ctx.fwd_tracker_states)
        detached = detach_variable(inputs)
        with torch.enable_grad():
            outputs = ctx.run_function(*detached)
        torch.set_rng_state(cpu_state)
        _dev_set_state(dev_state)
        get_cuda_rng_tracker().set_states(tracker)
        if isinstance(outputs, torch.Tensor):
            outputs = (outputs,)
        torch.autograd.backward(outputs, grads)
        return (None, None) + tuple(x.grad if isinstance(x, torch.Tensor) else None for x in detached)


def checkpoint(function, distribute_saved_activations, *args):
    return CheckpointFunction.apply(function, distribute_saved_activations, *args)
