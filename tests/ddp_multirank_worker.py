"""One rank of the multi-rank DDP race test (tests/test_ddp_multirank_gpu.py), launched by
torch.distributed.run. Every rank runs on cuda:0 over gloo (RCCL refuses two ranks on one GPU,
profiles/r4_rccl_two_ranks_one_gpu.txt), so the bucket collectives really combine gradients from
several processes while the producers run on the GPU.

Port of the reference's closed-form check (/root/reference/tests/distributed/ddp_race_condition_test.py:
21-22, 36-61): message_size=1 (one bucket per parameter), x filled with i + rank every iteration,
loss = sum((x * a) * b) so dL/da = x * b and dL/db = x * a, and after the average over ranks every
element must equal its closed form exactly — a bucket reduced before its gradient was written, a
copy-back that raced the consumer, or a stale bucket from the previous iteration shows up as a wrong
value. Random device sleeps in the backward reorder when the gradients become ready.

Prints one JSON line per rank: {"rank": r, "ok": bool, "mode": ..., "bad": [...]}.
"""
import argparse
import json
import os
import random
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


class _Delay(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cycles):
        ctx.cycles = cycles
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        if g.is_cuda:
            torch.cuda._sleep(ctx.cycles)
        return g, None


class Model(torch.nn.Module):
    """The reference's two-parameter model, plus n extra pairs of odd sizes (buckets straddling
    parameters when message_size > 1)."""

    def __init__(self, n, dtype, dev):
        super().__init__()
        self.a = torch.nn.Parameter(torch.full((n,), 1.0, device=dev, dtype=dtype))
        self.b = torch.nn.Parameter(torch.full((n,), 2.0, device=dev, dtype=dtype))
        self.extra = torch.nn.ParameterList(
            [torch.nn.Parameter(torch.full((1000 + 37 * i,), float(i % 3 + 1), device=dev, dtype=dtype))
             for i in range(12)])

    def forward(self, x, rng):
        out = ((_Delay.apply(self.a, rng.randint(0, 100000)) * x) * _Delay.apply(self.b, rng.randint(0, 100000))).sum()
        for i, p in enumerate(self.extra):
            out = out + _Delay.apply(p, rng.randint(0, 50000)).sum() * x[i]
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="default", choices=["default", "delay", "main_grad", "fp32_reduce"])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--numel", type=int, default=1 << 20)
    ap.add_argument("--device", default="cuda", help="cuda (every rank on cuda:0) or cpu (plumbing check)")
    args = ap.parse_args()
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    if args.device == "cuda":
        torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method="env://")
    from apex.parallel import DistributedDataParallel as DDP

    dtype = torch.bfloat16 if args.mode == "main_grad" else torch.float32
    torch.manual_seed(rank)
    net = Model(args.numel, dtype, args.device)
    kw = dict(message_size=1)
    if args.mode == "delay":
        kw = dict(delay_allreduce=True)
    elif args.mode == "main_grad":
        kw = dict(message_size=1, fp32_main_grad=True)
    elif args.mode == "fp32_reduce":
        kw = dict(message_size=3000, allreduce_always_fp32=True)
    model = DDP(net, **kw)
    x = torch.empty(args.numel, device=args.device, dtype=dtype)
    rng = random.Random(1234 + rank)  # different delays per rank: ranks reach the buckets out of step
    bad = []
    for i in range(args.iters):
        x.fill_(i + rank)  # fill x with new values every iteration
        model.zero_grad()  # (main_grad mode: also zero-fills the fp32 buffers)
        model(x, rng).backward()
        # closed form after the average over ranks: mean_r (i + r) = i + (world - 1) / 2
        xm = i + (world - 1) / 2.0

        def grad(p):
            return p.main_grad if args.mode == "main_grad" else p.grad

        checks = [("a", grad(net.a), 2.0 * xm), ("b", grad(net.b), 1.0 * xm)]
        # extra param e_i: d/de_i of sum(e_i) * x[i] = x[i] = i + rank  -> mean = xm
        checks += [("e%d" % j, grad(p), xm) for j, p in enumerate(net.extra)]
        for name, g, v in checks:
            if g is None:
                bad.append((i, name, "no grad"))
                continue
            want = torch.full_like(g, v)
            if not torch.equal(g, want):  # read on the default stream right after backward()
                bad.append((i, name, float((g.float() - want.float()).abs().max())))
    if args.device == "cuda":
        torch.cuda.synchronize()
    print(json.dumps({"rank": rank, "world": world, "mode": args.mode, "ok": not bad, "bad": bad[:8]}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
