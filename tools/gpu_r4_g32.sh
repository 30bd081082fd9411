#!/bin/bash
# round 4: Megatron GPT (fp32 main_grad on the transposed-read accumulate kernel) and ResNet-50 on the balanced-loop tree
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
T="timeout -k 10"
$T 500 python benchmarks/megatron_gpt.py --tp 1 --pp 1 --steps 4 --warmup 2 > $O/g32_megatron.json 2> $O/g32_megatron.err || exit 1
$T 300 python benchmarks/resnet50.py --steps 12 --warmup 4 > $O/g32_resnet50.json 2> $O/g32_resnet50.err || exit 1
for f in megatron resnet50; do python -c "import json;d=json.load(open('$O/g32_$f.json'));print('$f',d['value'],d['unit'],d['gpu']['timed']['sclk_mhz']['mean'] if 'gpu' in d else '')"; done
