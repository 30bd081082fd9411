#!/usr/bin/env python3
"""BASELINE.json config 1: 2-layer MLP, amp O0 (fp32 passthrough) + SGD on CPU, world_size=1.
A plumbing check: amp.initialize, scale_loss, the optimizer and the scaler run end to end and
the loss decreases. Reports samples/s and pass/fail.

  python benchmarks/mlp_cpu.py [--steps 50] [--warmup 5]
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    args = ap.parse_args()

    from apex import amp
    from apex.models.mlp import MLP, synthetic_batch
    from apex.utils.bench import emit, init_distributed, time_steps

    env = init_distributed(device="cpu")
    torch.manual_seed(0)
    model = MLP()
    opt = torch.optim.SGD(model.parameters(), lr=1e-3)
    model, opt = amp.initialize(model, opt, opt_level="O0", verbosity=0)
    x, y = synthetic_batch(args.batch)
    first = {}

    def step(i):
        opt.zero_grad()
        loss = F.mse_loss(model(x), y)
        with amp.scale_loss(loss, opt) as sl:
            sl.backward()
        opt.step()
        first.setdefault("loss", float(loss.detach()))
        return float(loss.detach())

    elapsed, last = time_steps(env, step, args.steps, args.warmup)
    emit(env, metric="2-layer MLP amp-O0 + SGD on CPU (plumbing)", items_per_step=args.batch, unit="samples/s",
         steps=args.steps, warmup=args.warmup, elapsed=elapsed, dtype="fp32", data="synthetic gaussian",
         config={"model": "MLP 1024-1024-16", "global_batch": args.batch, "parallelism": "none (CPU)"},
         extra={"pass": bool(last < first["loss"]), "first_loss": round(first["loss"], 5),
                "final_loss": round(last, 5)})


if __name__ == "__main__":
    main()
