#!/bin/bash
# round 4: the other BASELINE configurations on the current tree (GPT-2 1.5B, Megatron GPT
# 32L/H2560 TP1xPP1, ResNet-50 b256), MLM decoder vocab-padding microbench, optimizer stream
# timing
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
T="timeout -k 10"
$T 120 python tools/mlm_head_bench.py > $O/g11_mlm_head.jsonl 2> $O/g11_mlm_head.err || exit 1
$T 400 python benchmarks/gpt2.py --steps 6 --warmup 2 > $O/g11_gpt2.json 2> $O/g11_gpt2.err || exit 1
$T 500 python benchmarks/megatron_gpt.py --tp 1 --pp 1 --steps 4 --warmup 2 > $O/g11_megatron.json 2> $O/g11_megatron.err || exit 1
$T 300 python benchmarks/resnet50.py --steps 12 --warmup 4 > $O/g11_resnet50.json 2> $O/g11_resnet50.err || exit 1
$T 200 python tools/bw_kernels.py --ops adam,lamb --iters 10 > $O/g11_bw.jsonl 2> $O/g11_bw.err || exit 1
echo done
