#!/bin/bash
# round 4: fp32 flash kernels (tests, microbench vs the compositions), fp8 producer codes, bench
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
T="timeout -k 10"
PT="python -u -m pytest -q -x --timeout 120 --timeout-method thread"
$T 300 $PT tests/test_attention_f32_kernel_gpu.py tests/test_attention_fp32_gpu.py > $O/g7_f32_tests.log 2>&1 || exit 1
$T 300 $PT tests/test_fp8_gpu.py > $O/g7_fp8_tests.log 2>&1 || exit 1
$T 300 python tools/attn_f32_bench.py > $O/g7_attn_f32.jsonl 2> $O/g7_attn_f32.err || exit 1
$T 600 python bench.py --steps 10 --warmup 4 > $O/g7_bench.json 2> $O/g7_bench.err || exit 1
$T 600 python bench.py --steps 10 --warmup 4 --no-fp32 --fp8 > $O/g7_bench_fp8.json 2> $O/g7_bench_fp8.err || exit 1
echo done
