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


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def init_distributed(backend=None, device="cuda", single_rank_group=False):
    """Read RANK/WORLD_SIZE/LOCAL_RANK (torchrun), bind the GPU, init the process group.

    ``single_rank_group``: at WORLD_SIZE=1 still create a one-rank process group (RCCL on a GPU),
    so a data-parallel wrapper runs its hooks, bucket views and collectives at N=1 exactly as
    at N>1 (the 1-GPU line then measures the same code path as the scaling runs).

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
    elif world == 1 and single_rank_group and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if dev.type == "cuda" else "gloo"
        kw = {"device_id": dev} if (dev.type == "cuda" and backend == "nccl") else {}
        dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                                world_size=1, **kw)
    return DistEnv(rank, world, local_rank, dev)


def _sync(env):
    if env.device.type == "cuda":
        torch.cuda.synchronize()


def time_steps(env: DistEnv, step, steps: int, warmup: int, timer=None, sampler=None, on_timed_start=None):
    """Run ``step(i)`` warmup + steps times; return (max-over-ranks seconds, last result).

    ``timer`` (telemetry.StepTimer) records a HIP event between timed steps (no host sync);
    ``sampler`` (telemetry.GpuSampler) samples clocks/power while the timed steps run;
    ``on_timed_start`` runs after warmup, before the timed region (e.g. reset comm stats)."""
    out = None
    for i in range(warmup):
        out = step(i)
    _sync(env)
    if env.world > 1:
        dist.barrier()
    _sync(env)
    if on_timed_start is not None:
        on_timed_start()
    if sampler is not None:
        sampler.start()
    t0 = time.perf_counter()
    if timer is not None:
        timer.mark()
    for i in range(steps):
        out = step(i)
        if timer is not None:
            timer.mark()
    _sync(env)
    if env.world > 1:
        dist.barrier()
    _sync(env)
    elapsed = time.perf_counter() - t0
    if sampler is not None:
        sampler.stop()
    if env.world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=env.device if env.device.type == "cuda" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, out


def instrumented_steps(env: DistEnv, step, steps: int, warmup: int, ddp=None):
    """time_steps plus the run telemetry every benchmark line carries: per-step device time
    spread, GPU clocks / power / temperature during the timed steps (amdsmi), TunableOp state,
    library versions and, with an apex DDP wrapper, its bucket layout and comm timings.
    Returns (elapsed_s, last step result, extra dict)."""
    from . import telemetry

    timer = telemetry.StepTimer(enabled=env.device.type == "cuda")
    sampler = telemetry.GpuSampler(env.device.index or 0) if env.device.type == "cuda" else None
    idle = sampler.snapshot() if sampler is not None else None
    reset = ddp.reset_comm_stats if ddp is not None and hasattr(ddp, "reset_comm_stats") else None
    elapsed, out = time_steps(env, step, steps, warmup, timer=timer if timer.enabled else None,
                              sampler=sampler, on_timed_start=reset)
    extra = {"step_ms": timer.summary() if timer.enabled else None,
             "gpu": {"idle": idle, "timed": sampler.summary() if sampler is not None else None},
             "tunableop": telemetry.tunableop_status() if env.device.type == "cuda" else None,
             "versions": telemetry.library_versions()}
    if ddp is not None and hasattr(ddp, "comm_stats"):
        extra["ddp"] = ddp.comm_stats()
    if env.device.type == "cuda":
        extra["peak_mem_gb"] = round(torch.cuda.max_memory_allocated(env.device) / 2 ** 30, 1)
    return elapsed, out, extra


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


def max_over_ranks(env: DistEnv, value: float) -> float:
    if env.world > 1:
        t = torch.tensor([value], dtype=torch.float64,
                         device=env.device if env.device.type == "cuda" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())
    return value


def finish(env: DistEnv):
    if dist.is_initialized():
        dist.destroy_process_group()
