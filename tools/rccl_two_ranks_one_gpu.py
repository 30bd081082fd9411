"""Two RCCL ranks on ONE GPU: does the "nccl" (RCCL) backend run the multi-rank collective path
(ring setup, all-reduce / reduce-scatter / all-gather, apex DDP buckets) when both ranks share the
box's single MI355X? Used to exercise apex.parallel's N > 1 code on RCCL without an 8-GPU node.

  python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29511 tools/rccl_two_ranks_one_gpu.py

Rank 0 prints one JSON line (or the error RCCL raised).
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    out = {"world": world}
    try:
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
        x = torch.full((1 << 20,), float(rank + 1), device="cuda")
        dist.all_reduce(x)
        torch.cuda.synchronize()
        out["all_reduce_ok"] = bool(torch.all(x == sum(range(1, world + 1))).item())
        shards = torch.arange(world * 4, dtype=torch.float32, device="cuda")
        part = torch.empty(4, device="cuda")
        dist.reduce_scatter_tensor(part, shards)
        out["reduce_scatter_ok"] = bool(torch.equal(part.cpu(), world * torch.arange(rank * 4, rank * 4 + 4).float()))
        full = torch.empty(world * 4, device="cuda")
        dist.all_gather_into_tensor(full, part)
        out["all_gather_ok"] = bool(torch.equal(full.cpu(), world * torch.arange(world * 4).float()))

        # apex DDP on RCCL: several buckets, overlapped reduction, then a check that both ranks
        # hold identical averaged gradients
        from apex.parallel import DistributedDataParallel as DDP

        torch.manual_seed(0)
        model = torch.nn.Sequential(*[torch.nn.Linear(256, 256) for _ in range(6)]).cuda()
        ddp = DDP(model, message_size=256 * 256 * 2)
        torch.manual_seed(100 + rank)
        xin = torch.randn(32, 256, device="cuda")
        ddp(xin).square().mean().backward()
        torch.cuda.synchronize()
        flat = torch.cat([p.grad.flatten() for p in model.parameters()])
        ref = flat.clone()
        dist.all_reduce(ref)
        ref /= world
        gathered = [torch.empty_like(flat) for _ in range(world)]
        dist.all_gather(gathered, flat)
        out["ddp_grads_identical_across_ranks"] = all(torch.equal(gathered[0], g) for g in gathered)
        out["ddp_grads_are_average"] = bool(torch.allclose(flat, ref, rtol=1e-5, atol=1e-6))
        # bandwidth sample (shared GPU: NOT an xGMI number, both ranks on one device)
        y = torch.ones(64 << 20, device="cuda", dtype=torch.bfloat16)
        dist.all_reduce(y)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            dist.all_reduce(y)
        torch.cuda.synchronize()
        out["allreduce_128MB_bf16_ms_same_gpu"] = round((time.perf_counter() - t0) / 5 * 1e3, 3)
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report what RCCL said instead of a traceback per rank
        out["error"] = f"{type(e).__name__}: {e}"[:500]
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
