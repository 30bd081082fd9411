"""Metric plumbing (K-10 and the logging plan of SURVEY §5).

``reduce_tensor`` is the ImageNet example's scalar all-reduce
(reference examples/imagenet/main.py:485-489: clone, all_reduce SUM, divide by world).
``reduce_scalars`` packs several per-iteration scalars into ONE collective instead of
one latency-bound RCCL call each (loss, prec@1, prec@5 in the reference's loop).
"""
from __future__ import annotations

import json
import os
import time

import torch
import torch.distributed as dist


def _world(group=None):
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def reduce_tensor(tensor, group=None):
    rt = tensor.clone()
    ws = _world(group)
    if ws > 1:
        dist.all_reduce(rt, op=dist.ReduceOp.SUM, group=group)
    return rt / ws


def reduce_scalars(*values, group=None, device=None):
    """Average several scalars (python numbers or 0-d/1-element tensors) across ranks with a
    single all-reduce; returns a tuple of python floats."""
    if device is None:
        device = next((v.device for v in values if torch.is_tensor(v)), torch.device("cpu"))
        if dist.is_initialized() and dist.get_backend(group) == "nccl" and device.type != "cuda":
            device = torch.device("cuda", torch.cuda.current_device())
    buf = torch.stack([(v.detach().reshape(()).float() if torch.is_tensor(v) else torch.tensor(float(v)))
                       .to(device) for v in values])
    buf = reduce_tensor(buf, group)
    return tuple(float(x) for x in buf.cpu())


class AverageMeter:
    """Running average (reference examples/imagenet/main.py AverageMeter)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = 0.0
        self.avg = 0.0
        self.sum = 0.0
        self.count = 0

    def update(self, val, n=1):
        self.val = float(val)
        self.sum += float(val) * n
        self.count += n
        self.avg = self.sum / self.count


class JsonlLogger:
    """Rank-0 JSON-lines metrics writer (step time, throughput, loss, loss scale, ...)."""

    def __init__(self, path, rank=None):
        self.rank = (dist.get_rank() if dist.is_initialized() else 0) if rank is None else rank
        self.path = path
        self._f = None
        if self.rank == 0 and path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            self._f = open(path, "a")

    def log(self, **fields):
        if self._f is None:
            return
        fields.setdefault("time", time.time())
        self._f.write(json.dumps({k: (float(v) if torch.is_tensor(v) else v) for k, v in fields.items()}) + "\n")
        self._f.flush()

    def close(self):
        if self._f is not None:
            self._f.close()
            self._f = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
