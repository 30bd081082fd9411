#!/usr/bin/env python3
"""BASELINE.json config 4: GPT-2 1.5B (48L, H1600, 25 heads, seq 1024) with the apex.contrib
fused attention + xentropy, amp O2 bf16 + FusedAdam, apex DDP when N>1; tokens/s (whole job).
Synthetic token ids, random-init weights.

  python benchmarks/gpt2.py [--batch 8] [--seq 1024] [--steps 10] [--warmup 3]
  torchrun --nproc-per-node N benchmarks/gpt2.py ...
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    # per-GPU batch 16: measured 66.5k (b8) / 70.5k (b16) / 71.3k (b32) tokens/s on one MI355X
    # (profiles/r1_gpt2_batch_sweep.json); b16 keeps the step near 0.23 s
    ap.add_argument("--batch", type=int, default=16, help="per-GPU sequences")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", default="1.5b", choices=["1.5b", "medium", "tiny"])
    args = ap.parse_args()

    from apex.utils.bench import emit, finish, init_distributed, instrumented_steps
    from apex.utils.gemm_tuning import enable_tuned_gemms

    enable_tuned_gemms()

    env = init_distributed(single_rank_group=True)  # apex DDP at every N (hooks + buckets timed at N=1 too)
    import apex
    from apex import amp
    from apex.models.gpt import GPTConfig, GPTModel, param_groups, synthetic_batch
    from apex.optimizers import FusedAdam
    from apex.parallel import DistributedDataParallel as DDP

    apex._ext.require()
    torch.manual_seed(0)
    cfg = {"1.5b": GPTConfig.gpt2_1_5b, "medium": GPTConfig.gpt2_medium, "tiny": GPTConfig.tiny}[args.size]()
    model = GPTModel(cfg).to(env.device)
    opt = FusedAdam(param_groups(model, 0.1), lr=1.5e-4, betas=(0.9, 0.95), eps=1e-8)
    model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16, verbosity=0)
    model = DDP(model, message_size=int(os.environ.get("APEX_DDP_MESSAGE_SIZE", 25_000_000)), comm_timing=True)
    g = torch.Generator(device=env.device).manual_seed(1 + env.rank)
    batches = [synthetic_batch(cfg, args.batch, args.seq, device=env.device, generator=g) for _ in range(2)]

    def step(i):
        loss = model(**batches[i % 2])
        with amp.scale_loss(loss, opt) as sl:
            sl.backward()
        opt.step()
        opt.zero_grad()
        return loss

    elapsed, loss, extra = instrumented_steps(env, step, args.steps, args.warmup, ddp=model)
    nparams = sum(p.numel() for p in model.module.parameters())
    emit(env, metric="tokens/s GPT-2 1.5B fused multihead_attn + xentropy, amp-O2 bf16 + FusedAdam, DDP",
         items_per_step=args.batch * args.seq * env.world, unit="tokens/s", steps=args.steps,
         warmup=args.warmup, elapsed=elapsed, dtype="bf16", data="synthetic token ids; random-init weights",
         config={"model": f"GPT-2 {args.size} ({cfg.n_layer}L, H{cfg.n_embd}, {cfg.n_head} heads, "
                          f"{nparams / 1e9:.2f}B params)",
                 "global_batch": args.batch * env.world, "seq_len": args.seq, "parallelism": f"dp{env.world}"},
         extra=dict(extra, final_loss=round(float(loss), 4)))
    finish(env)


if __name__ == "__main__":
    main()
