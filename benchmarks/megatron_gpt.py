#!/usr/bin/env python3
"""BASELINE.json config 5: Megatron-style GPT on apex.transformer, TP x PP (x DP) over RCCL;
tokens/s for the whole job. 1F1B pipeline schedule, vocab-parallel embedding + CE, tied
embedding grads synced over the embedding group, amp O2 bf16 + FusedAdam.

  torchrun --nproc-per-node 8 benchmarks/megatron_gpt.py --tp 4 --pp 2      (config 5)
  python benchmarks/megatron_gpt.py --tp 1 --pp 1 --layers 8                 (1-GPU smoke)
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=4)
    ap.add_argument("--pp", type=int, default=2)
    ap.add_argument("--hidden", type=int, default=2560)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--heads", type=int, default=20, help="head dim 128 (2560/20) runs the MFMA flash kernel")
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--micro-batch", type=int, default=4)
    ap.add_argument("--global-batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--bf16-grad-accum", action="store_true",
                    help="accumulate micro-batch gradients in bf16 .grad (the pre-r3 path) instead of "
                         "the fp32 main_grad buffers")
    args = ap.parse_args()

    from apex.utils.bench import emit, finish, init_distributed, instrumented_steps
    from apex.utils.gemm_tuning import enable_tuned_gemms

    enable_tuned_gemms()

    env = init_distributed(single_rank_group=True)  # parallel_state needs a process group at N=1 too
    import torch.distributed as dist

    import apex
    from apex import amp
    from apex.models.megatron_gpt import (MegatronGPTConfig, build_stage, sync_embedding_grads,
                                          sync_initial_embeddings)
    from apex.optimizers import FusedAdam
    from apex.parallel import DistributedDataParallel as DDP
    from apex.transformer import parallel_state as ps
    from apex.transformer import tensor_parallel as tp
    from apex.transformer.pipeline_parallel import get_forward_backward_func, setup_microbatch_calculator

    apex._ext.require()
    if env.world == 1:
        args.tp = args.pp = 1
    ps.initialize_model_parallel(args.tp, args.pp)
    dp = ps.get_data_parallel_world_size()
    setup_microbatch_calculator(env.rank, None, args.global_batch, args.micro_batch, dp)
    torch.manual_seed(0)
    tp.model_parallel_cuda_manual_seed(1234)
    cfg = MegatronGPTConfig(hidden_size=args.hidden, num_layers=args.layers, num_attention_heads=args.heads,
                            max_position_embeddings=args.seq)
    model = build_stage(cfg).to(env.device)
    sync_initial_embeddings(model)
    opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01)
    model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16, verbosity=0)
    # data-parallel gradient reduction on apex DDP buckets over the DP group; the pipeline schedule
    # keeps the hooks off (no_sync) until each chunk's last microbatch backward, whose bucket
    # all-reduces then overlap it
    # micro-batch gradients accumulate in fp32 main_grad buffers (the weight-gradient GEMMs add
    # their fp32 result straight in; Megatron's main_grad) — no bf16 rounding per micro-batch, no
    # separate bf16 grad-add kernels
    model = DDP(model, message_size=int(os.environ.get("APEX_DDP_MESSAGE_SIZE", 25_000_000)),
                process_group=ps.get_data_parallel_group(), comm_timing=True,
                fp32_main_grad=not args.bf16_grad_accum)
    stage = model.module
    n_local = args.global_batch // dp
    g = torch.Generator(device=env.device).manual_seed(7 + ps.get_data_parallel_rank())
    ids = torch.randint(0, cfg.vocab_size, (n_local, args.seq), device=env.device, generator=g)
    fb = get_forward_backward_func(None, args.pp)

    def fwd_step(batch, m):
        out = m(batch, batch if ps.is_pipeline_last_stage() else None)
        return out, (lambda o: (o, {"loss": o.detach()}))

    def step(i):
        losses = fb(fwd_step, ids, model, forward_only=False,
                    tensor_shape=(args.micro_batch, args.seq, args.hidden), dtype=torch.bfloat16)
        sync_embedding_grads(stage)
        opt.step()
        opt.zero_grad()
        return losses

    elapsed, losses, extra = instrumented_steps(env, step, args.steps, args.warmup, ddp=model)
    loss = float(torch.stack([l["loss"] for l in losses]).float().mean()) if losses else None
    emit(env, metric="tokens/s Megatron-style GPT apex.transformer TP x PP over RCCL",
         items_per_step=args.global_batch * args.seq, unit="tokens/s", steps=args.steps, warmup=args.warmup,
         elapsed=elapsed, dtype="bf16", data="synthetic token ids; random-init weights",
         config={"model": f"GPT {args.layers}L H{args.hidden} {args.heads} heads", "global_batch": args.global_batch,
                 "micro_batch": args.micro_batch, "seq_len": args.seq,
                 "parallelism": f"tp{args.tp}xpp{args.pp}xdp{dp}",
                 "grad_accumulation": "bf16 .grad" if args.bf16_grad_accum else "fp32 main_grad"},
         extra=dict(extra, final_loss_last_stage_rank=loss))
    finish(env)


if __name__ == "__main__":
    main()
