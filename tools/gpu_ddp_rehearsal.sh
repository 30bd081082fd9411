#!/bin/bash
# Multi-rank rehearsal on ONE GPU: 2 ranks (gloo, both bound to cuda:0) through bench.py's DDP path
# (apex DDP bucket hooks + async all-reduce + FusedLAMB + amp O2) and the GPT-2 / ResNet benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
O=gpurun_out/${OUT:-ddp}
mkdir -p $O
export PYTHONUNBUFFERED=1 APEX_DIST_BACKEND=gloo APEX_DIST_SHARE_GPU=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps 4 --warmup 2 --layers 2 --batch 32 > $O/bert2.json 2> $O/bert2.err || { tail -30 $O/bert2.err; exit 4; }
cat $O/bert2.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
  benchmarks/resnet50.py --steps 3 --warmup 1 --batch 16 > $O/rn2.json 2> $O/rn2.err || { tail -30 $O/rn2.err; exit 5; }
cat $O/rn2.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 \
  benchmarks/gpt2.py --size tiny --steps 3 --warmup 1 --batch 2 --seq 128 > $O/gpt2.json 2> $O/gpt2.err || { tail -30 $O/gpt2.err; exit 6; }
cat $O/gpt2.json
for cfg in "2 1" "1 2"; do set -- $cfg
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2952$1 \
    benchmarks/megatron_gpt.py --tp $1 --pp $2 --hidden 512 --layers 4 --heads 4 --seq 256 --micro-batch 2 --global-batch 8 \
    --steps 2 --warmup 1 > $O/meg_tp$1_pp$2.json 2> $O/meg_tp$1_pp$2.err || { tail -30 $O/meg_tp$1_pp$2.err; exit 7; }
  cat $O/meg_tp$1_pp$2.json
done
echo "all done"
