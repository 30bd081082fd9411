"""Multi-GPU pre-flight and DDP bucket sizing for a data-parallel job (RCCL over xGMI).

A first 8-GPU run that fails or scales badly should say why on its first line. Three pieces,
all collective over the job's data-parallel group (every rank calls them at the same point):

* ``preflight_allreduce(group, device)`` — an all-reduce of KNOWN values in every dtype the DDP
  buckets use (rank r contributes r + 1, plus a per-element ramp so a rotated or truncated
  buffer is caught) with SUM and AVG; any mismatch raises on every rank with the rank count,
  expected and observed values. It also times one small message (latency) so the JSON line
  records what the communicator delivered before any training work ran.
* ``rccl_env()`` — the RCCL knobs in force (``NCCL_MIN/MAX_NCHANNELS``, algorithm / protocol
  overrides, ``APEX_DDP_CHANNELS``). On CDNA, RCCL's kernels occupy CUs: every channel is a
  workgroup that the backward GEMMs cannot use, so the channel cap trades all-reduce bandwidth
  against GEMM throughput while the two overlap. ``apply_channel_cap()`` turns
  ``APEX_DDP_CHANNELS=k`` into ``NCCL_MAX_NCHANNELS=k`` before the communicators are created.
* ``probe_bucket_sizes`` + ``select_bucket_sizes`` — time 2-3 candidate bucket sizes on the DDP
  communicator (MAX over ranks, so every rank picks the same) and choose the SMALLEST size
  whose bus bandwidth is within ``tolerance`` of the best: the smallest bucket that already
  saturates the xGMI ring keeps the most all-reduce work overlapped with backward (the last
  bucket, which cannot overlap, is at most one bucket). The first bucket (the gradients that
  arrive first in backward) is a quarter of that, so communication starts early.

Reference anchors: the reference's fixed ``message_size=10000000`` and side-stream all-reduce
(``/root/reference/apex/parallel/distributed.py:124,144,294-298``) and its rank-0 layout
broadcast (``:176-203``) — these helpers choose and check what the reference hard-codes.
"""
from __future__ import annotations

import os
import time

import torch
import torch.distributed as dist

_RCCL_VARS = ("NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS", "NCCL_ALGO", "NCCL_PROTO", "NCCL_P2P_LEVEL",
              "NCCL_NCHANNELS_PER_NET_PEER", "RCCL_MSCCL_ENABLE", "APEX_DDP_CHANNELS", "HSA_ENABLE_IPC_MODE_LEGACY")


def apply_channel_cap():
    """``APEX_DDP_CHANNELS=k`` -> ``NCCL_MAX_NCHANNELS=k`` (unless already set). Must run before
    the first communicator is created (i.e. before init_process_group with a device_id)."""
    k = os.environ.get("APEX_DDP_CHANNELS")
    if k and "NCCL_MAX_NCHANNELS" not in os.environ:
        os.environ["NCCL_MAX_NCHANNELS"] = str(int(k))
    return k


def rccl_env():
    return {k: os.environ.get(k) for k in _RCCL_VARS if os.environ.get(k) is not None}


class PreflightError(RuntimeError):
    pass


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def preflight_allreduce(group=None, device=None, numel=1 << 16, dtypes=(torch.bfloat16, torch.float32)):
    """All-reduce known values over ``group``; raise PreflightError on any mismatch.

    Rank r contributes ``(r + 1) + ramp`` with ``ramp[i] = i % 7`` (exact in bf16): SUM must give
    ``n(n+1)/2 + n * ramp`` and AVG ``(n+1)/2 + ramp``. Returns a dict for the result line."""
    device = torch.device(device) if device is not None else torch.device("cpu")
    n = dist.get_world_size(group)
    r = dist.get_rank(group)
    ramp = (torch.arange(numel, device=device) % 7).float()
    out = {"nranks": n, "ok": True, "checked": []}
    use_avg = dist.get_backend(group) == "nccl"  # gloo has no AVG
    bads, notes = [], []
    for dt in dtypes:
        ops = [("sum", dist.ReduceOp.SUM)] + ([("avg", dist.ReduceOp.AVG)] if use_avg else [])
        for name, op in ops:
            x = ((r + 1) + ramp).to(dt)
            dist.all_reduce(x, op=op, group=group)
            want = (n * (n + 1) / 2 + n * ramp) if name == "sum" else ((n + 1) / 2 + ramp)
            err = (x.float() - want).abs()
            tol = 0.0 if dt == torch.float32 else 0.02 * float(want.abs().max())
            bad = int((err > tol).sum())
            bads.append(bad)
            if bad:
                i = int(err.argmax())
                notes.append(f"({name}, {str(dt).replace('torch.', '')}): {bad}/{numel} wrong, e.g. [{i}] = "
                             f"{float(x[i].float()):g} vs {float(want[i]):g}")
            out["checked"].append(f"{name}:{str(dt).replace('torch.', '')}")
    # every rank learns every rank's verdict (one more tiny collective), so all ranks fail together
    # instead of the good ones hanging in the next collective
    mine = torch.tensor(bads, dtype=torch.float64, device=device)
    every = [torch.zeros_like(mine) for _ in range(n)]
    dist.all_gather(every, mine, group=group)
    failed = [i for i, t in enumerate(every) if float(t.sum()) > 0]
    if failed:
        raise PreflightError(
            f"pre-flight all-reduce over {n} ranks FAILED: group ranks {failed} received wrong results"
            + (f"; this rank (global {dist.get_rank()}): " + "; ".join(notes) if notes else "")
            + "; check RCCL / xGMI (rocm-smi --showtopo) and HSA_ENABLE_IPC_MODE_LEGACY=0")
    # small-message latency (8 KB), MAX over ranks
    small = torch.ones(4096, dtype=torch.bfloat16, device=device)
    for _ in range(3):
        dist.all_reduce(small, group=group)
    _sync(device)
    t0 = time.perf_counter()
    for _ in range(10):
        dist.all_reduce(small, group=group)
    _sync(device)
    out["small_allreduce_us"] = round(_max_over(group, (time.perf_counter() - t0) / 10, device) * 1e6, 1)
    out["rccl_env"] = rccl_env()
    return out


def _max_over(group, value, device):
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def probe_bucket_sizes(group=None, device=None, sizes=(8_000_000, 25_000_000, 50_000_000), dtype=torch.bfloat16,
                       iters=4):
    """Time one all-reduce per candidate bucket size (elements) on ``group``; MAX over ranks.
    Returns [{"numel", "us", "busbw_gbs"}] in ``sizes`` order."""
    device = torch.device(device) if device is not None else torch.device("cpu")
    n = dist.get_world_size(group)
    res = []
    for numel in sizes:
        buf = torch.ones(int(numel), dtype=dtype, device=device)
        dist.all_reduce(buf, group=group)
        _sync(device)
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(buf, group=group)
        _sync(device)
        t = _max_over(group, (time.perf_counter() - t0) / iters, device)
        nbytes = int(numel) * buf.element_size()
        bus = nbytes / t / 1e9 * 2 * (n - 1) / max(n, 1)
        res.append({"numel": int(numel), "us": round(t * 1e6, 1), "busbw_gbs": round(bus, 2)})
        del buf
    return res


def select_bucket_sizes(probe, tolerance=0.9, first_fraction=0.25, min_first=1_000_000):
    """(message_size, first_bucket_size) from a ``probe_bucket_sizes`` result: the smallest
    probed size reaching ``tolerance`` x the best bus bandwidth; the first bucket a
    ``first_fraction`` of it (at least ``min_first`` elements). Pure function (unit-tested)."""
    if not probe:
        raise ValueError("empty probe")
    best = max(p["busbw_gbs"] for p in probe)
    ok = sorted((p for p in probe if p["busbw_gbs"] >= tolerance * best), key=lambda p: p["numel"])
    msg = ok[0]["numel"]
    first = max(min_first, int(msg * first_fraction))
    return msg, min(first, msg)
