"""Shared benchmark harness (NS-09): one process per GPU, torch.distributed over RCCL,
W untimed warmup steps, K timed steps bracketed by barrier + device synchronize on both
sides, MAX elapsed over ranks, one JSON line from rank 0.

The headline ``bench.py`` and every ``benchmarks/*.py`` workload script use the same
timing contract, so numbers across configs are comparable.
"""
from __future__ import annotations

import json
import os
import sys
import time
from dataclasses import dataclass

import torch
import torch.distributed as dist


def log(*a):
    print(*a, file=sys.stderr, flush=True)


_RESULT_STREAM = None


def protect_stdout():
    """Reserve the process's stdout for the one JSON result line.

    Native libraries print banners to fd 1 (RCCL prints its version block on communicator
    init), which would break the one-line contract; fd 1 is pointed at stderr for the rest of
    the process and the original stdout is kept for :func:`emit`. Idempotent."""
    global _RESULT_STREAM
    if _RESULT_STREAM is None:
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        _RESULT_STREAM = os.fdopen(saved, "w", buffering=1)
    return _RESULT_STREAM


@dataclass
class DistEnv:
    rank: int
    world: int
    local_rank: int
    device: torch.device

    @property
    def is_main(self):
        return self.rank == 0


def init_distributed(backend=None, device="cuda"):
    """Read RANK/WORLD_SIZE/LOCAL_RANK (torchrun), bind the GPU, init the process group.

    Rehearsal knobs (not for measurements): ``APEX_DIST_BACKEND`` overrides the backend
    (e.g. ``gloo``), ``APEX_DIST_SHARE_GPU=1`` binds every rank to device 0, so the multi-rank
    path (DDP hooks, bucket all-reduces, metric reductions) runs on a one-GPU box."""
    protect_stdout()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("APEX_DIST_BACKEND") or backend
    if device == "cuda":
        dev_index = 0 if os.environ.get("APEX_DIST_SHARE_GPU", "0") == "1" else local_rank
        torch.cuda.set_device(dev_index)
        dev = torch.device("cuda", dev_index)
    else:
        dev = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if dev.type == "cuda" else "gloo"
        kw = {"device_id": dev} if (dev.type == "cuda" and backend == "nccl") else {}
        dist.init_process_group(backend, **kw)
    return DistEnv(rank, world, local_rank, dev)


def _sync(env):
    if env.device.type == "cuda":
        torch.cuda.synchronize()


def time_steps(env: DistEnv, step, steps: int, warmup: int):
    """Run ``step(i)`` warmup + steps times; return (max-over-ranks seconds, last result)."""
    out = None
    for i in range(warmup):
        out = step(i)
    _sync(env)
    if env.world > 1:
        dist.barrier()
    _sync(env)
    t0 = time.perf_counter()
    for i in range(steps):
        out = step(i)
    _sync(env)
    if env.world > 1:
        dist.barrier()
    _sync(env)
    elapsed = time.perf_counter() - t0
    if env.world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=env.device if env.device.type == "cuda" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, out


def emit(env: DistEnv, *, metric, items_per_step, unit, steps, warmup, elapsed, dtype, data, config,
         baseline=None, scaling="weak", extra=None):
    """Rank 0 prints the one-line JSON result; ``items_per_step`` is the whole-job count."""
    rate = items_per_step * steps / elapsed
    out = {
        "metric": metric,
        "value": round(rate, 3),
        "unit": unit,
        "n_gpus": env.world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(elapsed / steps * 1000.0, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None if baseline is None else round(rate / baseline, 4),
        "dtype": dtype,
        "data": data,
        "config": config,
    }
    if extra:
        out.update(extra)
    if env.is_main:
        stream = _RESULT_STREAM if _RESULT_STREAM is not None else sys.stdout
        print(json.dumps(out), file=stream, flush=True)
    return out


def finish(env: DistEnv):
    if env.world > 1 and dist.is_initialized():
        dist.destroy_process_group()
