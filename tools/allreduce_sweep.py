#!/usr/bin/env python3
"""All-reduce bus bandwidth vs message size over RCCL (xGMI) — picks apex DDP's bucket size.

One process per GPU (torchrun). For each dtype and message size: W warm-up and K timed
all-reduces (SUM) on a persistent buffer, timed with HIP events on the collective's stream and
max-reduced over ranks; reports algorithm bandwidth (bytes / t) and bus bandwidth
(algbw x 2(n-1)/n, the per-link figure a ring moves). Optionally runs C concurrent communicators
(``--comms``), each reducing its own buffer, the way ``DistributedDataParallel(num_allreduce_streams=C)``
overlaps buckets. The knee of the busbw curve is where a bucket is big enough to keep all of
RCCL's channels (spread over the 7 xGMI links of an MI355X node) busy; bigger buckets only delay
the first reduction in backward.

  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/allreduce_sweep.py [--min-mb 1 --max-mb 1024]
  (CPU / gloo rehearsal: APEX_DIST_BACKEND=gloo ... --cpu)
One JSON line per (dtype, size, comms) on rank 0's stdout.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-mb", type=float, default=1.0)
    ap.add_argument("--max-mb", type=float, default=1024.0)
    ap.add_argument("--dtypes", default="bf16,fp32")
    ap.add_argument("--comms", default="1,2", help="concurrent communicators to try")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args()
    from apex.utils.bench import init_distributed, protect_stdout

    env = init_distributed(device="cpu" if a.cpu else "cuda")
    out = protect_stdout()
    world = env.world
    dev = env.device
    comm_counts = [int(c) for c in a.comms.split(",")]
    groups = {1: [None]}
    for c in comm_counts:
        if c > 1:
            groups[c] = [dist.new_group(list(range(world))) for _ in range(c)]
    dts = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp16": torch.float16}
    sizes = []
    mb = a.min_mb
    while mb <= a.max_mb:
        sizes.append(mb)
        mb *= 2
    for dname in a.dtypes.split(","):
        dt = dts[dname]
        esz = torch.tensor([], dtype=dt).element_size()
        for mb in sizes:
            n = int(mb * 2 ** 20) // esz
            for c in comm_counts:
                bufs = [torch.ones(n // c, dtype=dt, device=dev) for _ in range(c)]
                streams = [torch.cuda.Stream() for _ in range(c)] if dev.type == "cuda" else [None] * c

                def once():
                    works = []
                    for b, g, s in zip(bufs, groups[c], streams):
                        if s is not None:
                            s.wait_stream(torch.cuda.current_stream())
                            with torch.cuda.stream(s):
                                works.append(dist.all_reduce(b, group=g, async_op=True))
                        else:
                            works.append(dist.all_reduce(b, group=g, async_op=True))
                    for w in works:
                        w.wait()

                for _ in range(a.warmup):
                    once()
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(a.iters):
                    once()
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                el = torch.tensor([(time.perf_counter() - t0) / a.iters], dtype=torch.float64, device=dev)
                dist.all_reduce(el, op=dist.ReduceOp.MAX)
                t = float(el.item())
                nbytes = (n // c) * c * esz
                algbw = nbytes / t / 1e9
                busbw = algbw * 2 * (world - 1) / world
                if env.rank == 0:
                    print(json.dumps({"dtype": dname, "size_mb": mb, "comms": c, "world": world,
                                      "backend": dist.get_backend(), "us": round(t * 1e6, 1),
                                      "algbw_gbs": round(algbw, 2), "busbw_gbs": round(busbw, 2)}), file=out, flush=True)
                del bufs
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
