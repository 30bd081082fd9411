#!/usr/bin/env python3
"""Headline benchmark: BERT-Large pre-training step, amp O2 (bf16) + FusedLAMB +
FusedLayerNorm + apex DistributedDataParallel (bucketed RCCL all-reduce).

BASELINE.json metric: "seq/sec BERT-Large amp-O2+FusedLAMB DDP at 1/2/4/8 MI355X; step
speedup vs fp32". Synthetic data of the real pre-training shapes, random-init weights
(no network access). Weak scaling: fixed per-GPU batch.

The model is wrapped in apex DDP at every N (at N=1 over a one-rank RCCL group), so the
gradient hooks, bucket views and bucket all-reduces are inside the timed region at 1 GPU too.

After the timed bf16 loop a second, shorter pass runs the SAME step in fp32 (amp O0, same
per-GPU batch: micro-batches of ``--fp32-microbatch`` accumulated, because fp32 activations
of 768 sequences do not fit) and reports ``speedup_vs_fp32`` = fp32 ms/step / bf16 ms/step —
the second half of the metric. ``--no-fp32`` skips it.

Usage:
  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--seq S] [--fp32-only]
  (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)
Rank 0 prints ONE JSON line on stdout.
"""
from __future__ import annotations

import argparse
import contextlib
import gc
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
    ap.add_argument("--fp32-only", action="store_true", help="time only the fp32 (amp O0) step")
    ap.add_argument("--no-fp32", action="store_true", help="skip the fp32 speedup pass")
    ap.add_argument("--fp32-steps", type=int, default=2)
    ap.add_argument("--fp32-microbatch", type=int, default=256)
    ap.add_argument("--layers", type=int, default=24, help="(debug only; the metric needs 24)")
    ap.add_argument("--fp8", action="store_true",
                    help="extra pass: the same step with amp fp8=True (NOT the headline: reported under extra.fp8); "
                         "on by default for a 1-GPU run")
    ap.add_argument("--no-fp8", action="store_true", help="skip the default 1-GPU fp8 pass")
    ap.add_argument("--fp8-steps", type=int, default=10)
    ap.add_argument("--fp16", action="store_true",
                    help="extra pass: the same step as amp O2 fp16 with DYNAMIC loss scaling (the reference's O2; "
                         "times the device-side overflow check / skip path; reported under extra.fp16)")
    ap.add_argument("--fp16-steps", type=int, default=10)
    # DDP bucket sizes (elements): at N>1 chosen by an in-job probe of the communicator unless
    # given here (apex.parallel.preflight.select_bucket_sizes); at N=1 there is no communication
    ap.add_argument("--message-size", type=int,
                    default=int(os.environ["APEX_DDP_MESSAGE_SIZE"]) if "APEX_DDP_MESSAGE_SIZE" in os.environ else None)
    ap.add_argument("--first-bucket-size", type=int, default=None)
    ap.add_argument("--ddp-fp32-allreduce", action="store_true",
                    help="reduce the bf16 gradient buckets in fp32 (A/B of the reduction precision)")
    ap.add_argument("--cpu-rehearsal", action="store_true",
                    help="REHEARSAL, not a measurement: the same N-rank sequence (pre-flight -> bucket probe -> "
                         "DDP -> timed steps -> max over ranks -> one JSON line) on CPU over gloo with a tiny "
                         "BERT, so the multi-GPU path is exercised where no GPUs are (tests/test_bench_rehearsal.py)")
    args = ap.parse_args()
    if args.cpu_rehearsal:
        os.environ.setdefault("APEX_DIST_BACKEND", "gloo")
        if "--batch" not in " ".join(sys.argv):
            args.batch = 8
        if "--seq" not in " ".join(sys.argv):
            args.seq = 32
        args.fp32_microbatch = min(args.fp32_microbatch, args.batch)
    return args


def build(env, cfg, fp32, message_size, fp8=False, first_bucket_size=None, fp32_allreduce=False,
          half=torch.bfloat16):
    from apex import amp
    from apex.amp._amp_state import _amp_state
    from apex.models.bert import BertForPreTraining, param_groups_for_lamb
    from apex.optimizers import FusedLAMB
    from apex.parallel import DistributedDataParallel as DDP

    _amp_state.optimizers, _amp_state.loss_scalers = [], []
    torch.manual_seed(1234)
    model = BertForPreTraining(cfg).to(env.device)
    opt = FusedLAMB(param_groups_for_lamb(model, 0.01), lr=6e-3, betas=(0.9, 0.999), eps=1e-6,
                    max_grad_norm=1.0)
    if fp32:
        model, opt = amp.initialize(model, opt, opt_level="O0", verbosity=0)
    else:
        kw = {"loss_scale": "dynamic"} if half == torch.float16 else {}
        model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=half, verbosity=0, fp8=fp8, **kw)
    model = DDP(model, message_size=message_size, first_bucket_size=first_bucket_size, comm_timing=True,
                allreduce_always_fp32=fp32_allreduce)
    return model, opt


def make_step(model, opt, batches, micro):
    from apex import amp

    def step(i):
        b = batches[i % len(batches)]
        n = b["input_ids"].shape[0]
        chunks = max(1, n // micro) if micro else 1
        loss = None
        for c in range(chunks):
            sub = {k: v[c * n // chunks:(c + 1) * n // chunks] for k, v in b.items()} if chunks > 1 else b
            last = c == chunks - 1
            ctx = model.no_sync() if not last else contextlib.nullcontext()
            with ctx:
                loss = model(**sub)
                with amp.scale_loss(loss / chunks if chunks > 1 else loss, opt,
                                    delay_unscale=not last) as scaled:
                    scaled.backward()
        opt.step()
        opt.zero_grad()
        return loss

    return step


def _sync(env):
    if env.device.type == "cuda":
        torch.cuda.synchronize()


def allreduce_probe(env, numel, iters=5):
    """Bus bandwidth of one DDP-bucket-sized bf16 all-reduce on this job's communicator (the
    scaling runs' diagnostic: compare with tools/allreduce_sweep.py's curve)."""
    import time

    import torch.distributed as dist

    buf = torch.ones(numel, dtype=torch.bfloat16, device=env.device)
    for _ in range(2):
        dist.all_reduce(buf)
    _sync(env)
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.all_reduce(buf)
    _sync(env)
    t = (time.perf_counter() - t0) / iters
    nbytes = numel * 2
    algbw = nbytes / t / 1e9
    return {"bytes": nbytes, "us": round(t * 1e6, 1), "algbw_gbs": round(algbw, 2),
            "busbw_gbs": round(algbw * 2 * (env.world - 1) / env.world, 2)}


def main():
    args = parse()
    from apex.utils import telemetry
    from apex.utils.bench import emit, finish, init_distributed, log, max_over_ranks, time_steps
    from apex.utils.gemm_tuning import DEFAULT_DIR, enable_tuned_gemms

    from apex.parallel import preflight

    rehearsal = args.cpu_rehearsal
    tuned = enable_tuned_gemms() if not rehearsal else False  # committed hipBLASLt/rocBLAS selections
    preflight.apply_channel_cap()  # APEX_DDP_CHANNELS -> NCCL_MAX_NCHANNELS, before any communicator
    # (also reserves stdout for the result line)
    env = init_distributed(single_rank_group=True, device="cpu" if rehearsal else "cuda")
    if env.world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={env.world}; using WORLD_SIZE")
    dev = env.device

    import apex
    from apex.models.bert import BertConfig, synthetic_batch

    if rehearsal:
        torch.set_num_threads(max(1, (os.cpu_count() or 2) // max(1, env.world)))
        cfg = BertConfig.tiny()
        args.layers = cfg.num_hidden_layers
    else:
        apex._ext.require()
        cfg = BertConfig.large()
        cfg.num_hidden_layers = args.layers
    world = env.world

    def batches_for(n):
        g = torch.Generator(device=dev)
        g.manual_seed(42 + env.rank)
        return [synthetic_batch(cfg, n, args.seq, device=dev, generator=g) for _ in range(4)]

    extra = {}
    # multi-GPU pre-flight: known-value all-reduces on the DDP communicator (fails loudly), the
    # RCCL settings in force, and the bucket sizes from an in-job probe of 3 candidate sizes
    dist_info = {"nranks": world, "rccl_env": preflight.rccl_env()}
    message_size, first_bucket = args.message_size, args.first_bucket_size
    if world > 1:
        dist_info["preflight"] = preflight.preflight_allreduce(None, dev)
        if message_size is None:
            # (rehearsal: CPU-sized candidates; the tiny model's whole gradient is ~1M elements)
            probe = preflight.probe_bucket_sizes(None, dev, sizes=(50_000, 100_000, 200_000)) if rehearsal \
                else preflight.probe_bucket_sizes(None, dev)
            message_size, auto_first = preflight.select_bucket_sizes(probe)
            first_bucket = first_bucket if first_bucket is not None else auto_first
            dist_info["bucket_probe"] = probe
            dist_info["bucket_choice"] = "probe (smallest size within 90% of the best bus bandwidth)"
        else:
            dist_info["bucket_choice"] = "flag"
    if message_size is None:
        message_size = 25_000_000
    dist_info.update(message_size=message_size, first_bucket_size=first_bucket,
                     allreduce_dtype="fp32" if args.ddp_fp32_allreduce else "bf16")
    extra["dist"] = dist_info
    args.message_size = message_size

    sampler = telemetry.GpuSampler(dev.index or 0) if not rehearsal else None
    idle = sampler.snapshot() if sampler is not None else None
    if not args.fp32_only:
        model, opt = build(env, cfg, False, args.message_size, first_bucket_size=first_bucket,
                           fp32_allreduce=args.ddp_fp32_allreduce)
        batches = batches_for(args.batch)
        timer = telemetry.StepTimer(enabled=not rehearsal)
        elapsed, loss = time_steps(env, make_step(model, opt, batches, 0), args.steps, args.warmup,
                                   timer=timer, sampler=sampler, on_timed_start=model.reset_comm_stats)
        final_loss = float(loss.float().item())
        ms = elapsed / args.steps * 1000.0
        extra["final_loss"] = round(final_loss, 4)
        extra["step_ms"] = timer.summary() if not rehearsal else None
        extra["ddp"] = model.comm_stats()
        if not rehearsal:
            extra["peak_mem_gb"] = round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 1)
        del model, opt, batches, loss
        gc.collect()
        if not rehearsal:
            torch.cuda.empty_cache()
    # the fp8 pass runs by default on one GPU (so the round-end record carries its speedup, not only
    # builder runs); multi-GPU runs keep it opt-in
    if (args.fp8 or (world == 1 and not args.no_fp8 and not rehearsal)) and not args.fp32_only:
        # per-tensor scaled fp8 forward / input-gradient GEMMs (apex.fp8): an extension beyond the
        # metric's amp O2 bf16 configuration, so it never replaces the headline value
        from apex import fp8 as _fp8

        def fp8_pass():
            if not rehearsal:
                torch.cuda.reset_peak_memory_stats(dev)
            model, opt = build(env, cfg, False, args.message_size, fp8=True)
            batches = batches_for(args.batch)
            f8_sampler = telemetry.GpuSampler(dev.index or 0) if not rehearsal else None
            f8_el, f8_loss = time_steps(env, make_step(model, opt, batches, 0), args.fp8_steps, 3,
                                        sampler=f8_sampler)
            f8_ms = max_over_ranks(env, f8_el / args.fp8_steps * 1000.0)
            extra["fp8"] = {"ms_per_step": round(f8_ms, 2), "seq_per_s": round(args.batch * world / f8_ms * 1000.0, 2),
                            "speedup_vs_bf16": round(ms / f8_ms, 3),
                            "final_loss": round(float(f8_loss.float().item()), 4),
                            "steps": args.fp8_steps, "recipe": "hybrid e4m3 fwd / e5m2 bwd, delayed scaling (history 16)",
                            "weight_grads": "bf16" if _fp8._FP8_WGRAD == "0" else "fp8 (e5m2 dy x e4m3 x, gemm_tt_f8)",
                            "codes_only_outputs": _fp8._FP8_CODES_ONLY != "0"}
            if not rehearsal:
                # clocks / power under the fp8 step (it runs at a higher clock than the bf16 step:
                # less power per token at the same 1400 W cap)
                extra["fp8"]["gpu"] = f8_sampler.summary()
                extra["fp8"]["peak_mem_gb"] = round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 1)

        if world == 1:
            # one GPU: an fp8 failure is reported in the line and never costs the headline
            try:
                fp8_pass()
            except Exception as e:  # noqa: BLE001
                extra["fp8"] = {"error": f"{type(e).__name__}: {e}"[:300]}
        else:
            fp8_pass()
        _fp8.disable()
        gc.collect()
        torch.cuda.empty_cache()
    if args.fp16 and not args.fp32_only:
        # amp O2 fp16 with dynamic loss scaling (reference semantics: /root/reference/apex/amp/scaler.py:20-55);
        # the overflow check + skip decision stay on the device (no host sync in the timed steps)
        from apex.amp._amp_state import _amp_state

        model, opt = build(env, cfg, False, args.message_size, first_bucket_size=first_bucket, half=torch.float16)
        batches = batches_for(args.batch)
        h_el, h_loss = time_steps(env, make_step(model, opt, batches, 0), args.fp16_steps, 3)
        h_ms = max_over_ranks(env, h_el / args.fp16_steps * 1000.0)
        sc = _amp_state.loss_scalers[0]
        extra["fp16"] = {"ms_per_step": round(h_ms, 2), "seq_per_s": round(args.batch * world / h_ms * 1000.0, 2),
                         "speedup_vs_bf16": round(ms / h_ms, 3) if not args.fp32_only else None,
                         "final_loss": round(float(h_loss.float().item()), 4),
                         "final_loss_scale": sc.loss_scale(), "steps": args.fp16_steps,
                         "config": "amp O2 fp16, dynamic loss scale (init 2^16, window 2000), FusedLAMB"}
        del model, opt, batches, h_loss
        gc.collect()
        torch.cuda.empty_cache()
    if world > 1 and not args.fp32_only:
        extra["allreduce_probe"] = allreduce_probe(env, args.message_size)
    fp32_ms = None
    if args.fp32_only or not args.no_fp32:
        model, opt = build(env, cfg, True, args.message_size)
        batches = batches_for(args.batch)
        f_el, _ = time_steps(env, make_step(model, opt, batches, args.fp32_microbatch),
                             max(1, args.fp32_steps), 1)
        fp32_ms = f_el / max(1, args.fp32_steps) * 1000.0
        del model, opt, batches
        gc.collect()
        if not rehearsal:
            torch.cuda.empty_cache()
    if args.fp32_only:
        elapsed, ms = f_el, fp32_ms
        steps = max(1, args.fp32_steps)
    else:
        steps = args.steps
        if fp32_ms is not None:
            fp32_ms = max_over_ranks(env, fp32_ms)
            extra["fp32_ms_per_step"] = round(fp32_ms, 2)
            extra["fp32_seq_per_s"] = round(args.batch * world / fp32_ms * 1000.0, 2)
            extra["speedup_vs_fp32"] = round(fp32_ms / ms, 3)
            extra["fp32_config"] = f"amp O0 fp32, micro-batches of {args.fp32_microbatch} accumulated to {args.batch}"
            from apex.contrib.multihead_attn import attention as _att

            d_head = cfg.hidden_size // cfg.num_attention_heads
            q = torch.empty(args.fp32_microbatch, args.seq, cfg.num_attention_heads, d_head, device="meta")
            if os.environ.get("APEX_ATTN_F32", "1") != "0" and d_head <= 128 and not rehearsal:
                path = "f32-MFMA flash kernels (csrc/attention_f32.hip)"
            elif _att._short_dense_ok(q, q, None):
                path = ("dense fp32 composition (fused softmax / dropout kernels, f32 MFMA GEMMs; "
                        "apex.contrib.multihead_attn.attention._fallback)")
            else:
                path = "query-blocked fp32 composition (apex.contrib.multihead_attn.chunked)"
            extra["fp32_attention_path"] = path + (
                "; history: round 3 sent this step through 16-row query blocks (2458 ms, which inflated "
                "its speedup_vs_fp32), round 4 first the dense composition (1558 ms), then the f32 kernels")
    if rehearsal:
        extra["rehearsal"] = ("CPU/gloo rehearsal of the N-rank bench sequence with a tiny BERT "
                              f"({cfg.num_hidden_layers}L H{cfg.hidden_size}): NOT a measurement")
    else:
        extra["gpu"] = {"idle": idle, "timed": sampler.summary()}
        tstat = telemetry.tunableop_status()
        tstat["committed_validators_match"] = None
        committed = telemetry.committed_validators(os.path.join(DEFAULT_DIR, "tunableop_results0.csv"))
        if committed and tstat.get("validators"):
            tstat["committed_validators_match"] = all(tstat["validators"].get(k) == v for k, v in committed.items())
        extra["tunableop"] = tstat
    extra["versions"] = telemetry.library_versions()
    emit(env, metric=METRIC, items_per_step=args.batch * world, unit="seq/s", steps=steps,
         warmup=args.warmup, elapsed=elapsed, baseline=BASELINE_VALUE, dtype="fp32" if args.fp32_only else "bf16",
         data="synthetic (random token ids, 15% masked positions, random NSP labels); random-init weights",
         config={
             "model": f"BERT-tiny REHEARSAL ({cfg.num_hidden_layers}L, H{cfg.hidden_size}; not the metric config)"
             if rehearsal else "BERT-Large (24L, H1024, A16, FFN4096, vocab 30522)" if args.layers == 24
             else f"BERT-Large-{args.layers}L (DEBUG, not the metric config)",
             "global_batch": args.batch * world,
             "per_gpu_batch": args.batch,
             "seq_len": args.seq,
             "max_predictions_per_seq": max(1, int(round(args.seq * 0.15))),
             "parallelism": f"dp{world}",
             "amp": "O0" if args.fp32_only else "O2 bf16",
             "optimizer": "FusedLAMB",
             "norm": "FusedLayerNorm",
             "ddp": f"apex.parallel.DistributedDataParallel ({'RCCL' if dev.type == 'cuda' else 'gloo'}, "
                    f"message_size {args.message_size})",
             "gemm_selection": "TunableOp pre-tuned (tuning/)" if tuned else "hipBLASLt default",
         },
         extra=extra)
    finish(env)


if __name__ == "__main__":
    main()
