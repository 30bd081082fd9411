#!/usr/bin/env python3
"""Headline benchmark: BERT-Large pre-training step, amp O2 (bf16) + FusedLAMB +
FusedLayerNorm + apex DistributedDataParallel (bucketed RCCL all-reduce).

BASELINE.json metric: "seq/sec BERT-Large amp-O2+FusedLAMB DDP at 1/2/4/8 MI355X; step
speedup vs fp32". Synthetic data of the real pre-training shapes, random-init weights
(no network access). Weak scaling: fixed per-GPU batch.

Usage:
  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--seq S] [--fp32]
  (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)
Rank 0 prints ONE JSON line on stdout.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

METRIC = "seq/sec BERT-Large amp-O2+FusedLAMB DDP at 1/2/4/8 MI355X; step speedup vs fp32"
BASELINE_VALUE = None  # BASELINE.json "published": {} -> no reference number


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    # per-GPU batch 768 (weak scaling): measured on MI355X (profiles/r1_bench_batch_sweep.json)
    # b256 3455, b384 3590, b512 3655-3665, b768 3729, b1024 3755 seq/s — larger GEMMs amortise
    # the epilogues and the fixed LAMB cost; 288 GB of HBM holds b768's activations easily
    ap.add_argument("--batch", type=int, default=int(os.environ.get("APEX_BENCH_BATCH", 768)),
                    help="per-GPU sequences per step")
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--fp32", action="store_true", help="fp32 (amp O0) reference run")
    ap.add_argument("--layers", type=int, default=24, help="(debug only; the metric needs 24)")
    ap.add_argument("--profile-steps", type=int, default=0)
    return ap.parse_args()


def main():
    args = parse()
    from apex.utils.bench import emit, finish, init_distributed, log, time_steps
    from apex.utils.gemm_tuning import enable_tuned_gemms

    tuned = enable_tuned_gemms()  # committed hipBLASLt/rocBLAS selections, read-only
    env = init_distributed()  # also reserves stdout for the result line
    if env.world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={env.world}; using WORLD_SIZE")
    dev = env.device

    import apex
    from apex import amp
    from apex.models.bert import BertConfig, BertForPreTraining, param_groups_for_lamb, synthetic_batch
    from apex.optimizers import FusedLAMB
    from apex.parallel import DistributedDataParallel as DDP

    apex._ext.require()
    torch.manual_seed(1234)
    cfg = BertConfig.large()
    cfg.num_hidden_layers = args.layers
    model = BertForPreTraining(cfg).to(dev)
    opt = FusedLAMB(param_groups_for_lamb(model, 0.01), lr=6e-3, betas=(0.9, 0.999), eps=1e-6,
                    max_grad_norm=1.0)
    if args.fp32:
        model, opt = amp.initialize(model, opt, opt_level="O0", verbosity=0)
    else:
        model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16,
                                    verbosity=0)
    if env.world > 1:
        model = DDP(model, message_size=int(os.environ.get("APEX_DDP_MESSAGE_SIZE", 25_000_000)))

    g = torch.Generator(device=dev)
    g.manual_seed(42 + env.rank)
    batches = [synthetic_batch(cfg, args.batch, args.seq, device=dev, generator=g) for _ in range(4)]

    def step(i):
        b = batches[i % len(batches)]
        loss = model(**b)
        with amp.scale_loss(loss, opt) as scaled:
            scaled.backward()
        opt.step()
        opt.zero_grad()
        return loss

    elapsed, loss = time_steps(env, step, args.steps, args.warmup)
    final_loss = float(loss.float().item())
    world = env.world
    emit(env, metric=METRIC, items_per_step=args.batch * world, unit="seq/s", steps=args.steps,
         warmup=args.warmup, elapsed=elapsed, baseline=BASELINE_VALUE, dtype="fp32" if args.fp32 else "bf16",
         data="synthetic (random token ids, 15% masked positions, random NSP labels); random-init weights",
         config={
             "model": "BERT-Large (24L, H1024, A16, FFN4096, vocab 30522)" if args.layers == 24
             else f"BERT-Large-{args.layers}L (DEBUG, not the metric config)",
             "global_batch": args.batch * world,
             "per_gpu_batch": args.batch,
             "seq_len": args.seq,
             "max_predictions_per_seq": max(1, int(round(args.seq * 0.15))),
             "parallelism": f"dp{world}",
             "amp": "O0" if args.fp32 else "O2 bf16",
             "optimizer": "FusedLAMB",
             "norm": "FusedLayerNorm",
             "ddp": "apex.parallel.DistributedDataParallel (RCCL)" if world > 1 else "none (1 GPU)",
             "gemm_selection": "TunableOp pre-tuned (tuning/)" if tuned else "hipBLASLt default",
         },
         extra={"final_loss": round(final_loss, 4)})
    finish(env)


if __name__ == "__main__":
    main()
