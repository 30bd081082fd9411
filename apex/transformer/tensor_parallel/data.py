"""Broadcast a batch from TP rank 0 to the rest of the TP group (one flattened collective)."""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import parallel_state as ps


def broadcast_data(keys, data, datatype):
    """Rank 0 of the TP group supplies ``data[key]``; every rank returns the same dict."""
    group = ps.get_tensor_model_parallel_group()
    src = ps.get_tensor_model_parallel_src_rank()
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    if ps.get_tensor_model_parallel_rank() == 0:
        sizes = []
        for k in keys:
            assert data[k].dtype == datatype, "{} has data type {} which is different than {}".format(
                k, data[k].dtype, datatype)
            sizes.append(len(data[k].shape))
            sizes.extend(data[k].shape)
        meta = torch.tensor([len(keys)] + sizes, dtype=torch.long, device=dev)
    else:
        meta = None
    n = torch.zeros(1, dtype=torch.long, device=dev) if meta is None else meta[:1].clone()
    dist.broadcast(n, src, group=group)
    mlen = torch.zeros(1, dtype=torch.long, device=dev) if meta is None else torch.tensor(
        [meta.numel()], dtype=torch.long, device=dev)
    dist.broadcast(mlen, src, group=group)
    if meta is None:
        meta = torch.zeros(int(mlen.item()), dtype=torch.long, device=dev)
    dist.broadcast(meta, src, group=group)
    m = meta.tolist()
    shapes, i = [], 1
    for _ in range(m[0]):
        nd = m[i]
        shapes.append(m[i + 1:i + 1 + nd])
        i += 1 + nd
    total = sum(int(torch.tensor(s).prod().item()) if s else 1 for s in shapes)
    if ps.get_tensor_model_parallel_rank() == 0:
        flat = torch.cat([data[k].contiguous().view(-1).to(dev) for k in keys])
    else:
        flat = torch.empty(total, dtype=datatype, device=dev)
    dist.broadcast(flat, src, group=group)
    out, off = {}, 0
    for k, s in zip(keys, shapes):
        numel = int(torch.tensor(s).prod().item()) if s else 1
        out[k] = flat[off:off + numel].view(s)
        off += numel
    return out
