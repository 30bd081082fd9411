#!/bin/bash
# round 4: multi-rank rehearsal on the one-GPU box (gloo, every rank on cuda:0): bench.py's N>1
# path at 2 and 4 ranks, ResNet-50 / GPT-2 / Megatron TP2 and PP2 through the same launcher
set -o pipefail
O=gpurun_out/r4/ddp; mkdir -p $O
OUT=r4/ddp bash tools/gpu_ddp_rehearsal.sh > $O/rehearsal.log 2>&1 || { tail -30 $O/rehearsal.log; exit 1; }
export PYTHONUNBUFFERED=1 APEX_DIST_BACKEND=gloo APEX_DIST_SHARE_GPU=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 \
  bench.py --gpus 4 --steps 3 --warmup 1 --layers 2 --batch 32 > $O/bert4.json 2> $O/bert4.err || { tail -30 $O/bert4.err; exit 2; }
cat $O/bert4.json | tail -c 600
echo done
