#!/bin/bash
# round 4: full GPU suite, bench (bf16 + fp32 pass), fp8 step kernel table
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -q -m gpu -x --timeout 120 --timeout-method thread tests/ > $O/g10_gpu_suite.log 2>&1 || exit 1
$T 600 python bench.py --steps 10 --warmup 4 > $O/g10_bench.json 2> $O/g10_bench.err || exit 1
OUT=r4/g10_fp8prof bash tools/gpu_fp8_prof.sh > $O/g10_fp8prof.log 2>&1 || exit 1
echo done
