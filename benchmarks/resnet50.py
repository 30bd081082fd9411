#!/usr/bin/env python3
"""BASELINE.json config 2: ResNet-50, amp O2 bf16 + FusedSGD + SyncBatchNorm (+ apex DDP when
N>1), img/s. Synthetic normalised images (NHWC/channels_last, MIOpen's fast bf16 layout) and
random-init weights. Throughput = world x batch / step time (the reference's definition,
examples/imagenet/main.py:348,354).

  python benchmarks/resnet50.py [--batch 256] [--steps 20] [--warmup 5] [--no-syncbn] [--no-fuse-bn] [--fp32]
  torchrun --nproc-per-node N benchmarks/resnet50.py ...
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-syncbn", action="store_true")
    ap.add_argument("--no-fuse-bn", action="store_true", help="BN, residual add and ReLU as separate ops")
    ap.add_argument("--graph", action="store_true",
                    help="replay the training step as a HIP graph (one process per GPU, N = 1 path)")
    ap.add_argument("--nchw", action="store_true", help="keep NCHW activations")
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--conv-search", action="store_true",
                    help="MIOpen Find (time every conv algorithm per shape in warmup) instead of immediate mode")
    args = ap.parse_args()
    # measured (profiles/r2_resnet50_conv_search_ab.json): the search gains nothing over MIOpen's
    # immediate-mode choice at this configuration (5775 vs 5816 img/s) and costs minutes of warmup
    torch.backends.cudnn.benchmark = args.conv_search

    from apex.utils.bench import emit, finish, init_distributed, instrumented_steps

    env = init_distributed(single_rank_group=True)  # apex DDP at every N (hooks + buckets timed at N=1 too)
    import apex
    from apex import amp
    from apex.models.resnet import fuse_bn_relu, resnet50, synthetic_batch
    from apex.optimizers import FusedSGD
    from apex.parallel import DistributedDataParallel as DDP
    from apex.parallel import convert_syncbn_model

    apex._ext.require()
    torch.manual_seed(0)
    model = resnet50()
    if not args.no_syncbn:
        model = convert_syncbn_model(model)  # channels_last inputs take the NHWC kernels
        if not args.no_fuse_bn:
            fuse_bn_relu(model)  # BN + residual add + ReLU as one HIP kernel each way
    cl = not args.nchw
    model = model.to(env.device, memory_format=torch.channels_last if cl else torch.contiguous_format)
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    if args.fp32:
        model, opt = amp.initialize(model, opt, opt_level="O0", verbosity=0)
    else:
        model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16, verbosity=0)
    model = DDP(model, message_size=int(os.environ.get("APEX_DDP_MESSAGE_SIZE", 25_000_000)),
                comm_timing=not args.graph)  # (timing events are not recorded inside a captured graph)
    g = torch.Generator(device=env.device).manual_seed(1 + env.rank)
    dt = torch.float32 if args.fp32 else torch.bfloat16
    batches = [synthetic_batch(args.batch, args.image_size, device=env.device, dtype=dt, channels_last=cl,
                               generator=g) for _ in range(2)]

    def step(i):
        x, y = batches[i % 2]
        loss = F.cross_entropy(model(x).float(), y)
        with amp.scale_loss(loss, opt) as sl:
            sl.backward()
        opt.step()
        opt.zero_grad()
        return loss

    run, graphed = step, False
    if args.graph:
        # the whole training step (forward, backward, loss scaling, FusedSGD) as one HIP graph per
        # input buffer, replayed each step: at ~2000 dispatches per step the eager loop leaves the
        # GPU idle ~13 % of the time between launches (profiles/r3_resnet50_step_kernels.txt).
        # Captured after eager warmup steps (MIOpen algorithm selection, the DDP bucket layout and
        # the optimizer state exist by then); any capture failure falls back to the eager step.
        try:
            for i in range(3):
                step(i)
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for i in range(2):
                    step(i)
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            graphs, outs = [], []
            for k in range(2):
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr):
                    outs.append(step(k))
                graphs.append(gr)

            def run(i):
                graphs[i % 2].replay()
                return outs[i % 2]

            graphed = True
        except Exception as e:  # noqa: BLE001
            print(f"graph capture failed, eager steps: {e!r}"[:300], file=sys.stderr)
            torch.cuda.synchronize()
    elapsed, loss, extra = instrumented_steps(env, run, args.steps, args.warmup, ddp=model)
    extra["hip_graph"] = graphed
    emit(env, metric="img/s ResNet-50 amp-O2 bf16 + FusedSGD + SyncBatchNorm", items_per_step=args.batch * env.world,
         unit="img/s", steps=args.steps, warmup=args.warmup, elapsed=elapsed,
         dtype="fp32" if args.fp32 else "bf16", data="synthetic normalised images; random-init weights",
         config={"model": "ResNet-50", "global_batch": args.batch * env.world, "image_size": args.image_size,
                 "parallelism": f"dp{env.world}", "syncbn": not args.no_syncbn,
                 "memory_format": "channels_last" if cl else "nchw"},
         extra=dict(extra, final_loss=round(float(loss), 4)))
    finish(env)


if __name__ == "__main__":
    main()
