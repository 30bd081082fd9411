#!/bin/bash
# round 4: fp8 producer-side codes from the flash kernels (tests + the bench's fp8 pass), plain-GEMM
# library reference
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
T="timeout -k 10"
PT="python -u -m pytest -q -x --timeout 120 --timeout-method thread"
$T 400 $PT tests/test_fp8_gpu.py tests/test_attention_gpu.py tests/test_attention_ext_gpu.py > $O/g5_tests.log 2>&1 || exit 1
$T 300 python tools/gemm_lib_ref.py > $O/g5_gemm_lib_ref.jsonl 2> $O/g5_gemm_lib_ref.err || exit 1
$T 600 python bench.py --steps 10 --warmup 4 --no-fp32 --fp8 > $O/g5_bench_fp8.json 2> $O/g5_bench_fp8.err || exit 1
APEX_FP8_PRODUCER=0 $T 600 python bench.py --steps 10 --warmup 4 --no-fp32 --fp8 > $O/g5_bench_fp8_noprod.json 2> $O/g5_bench_fp8_noprod.err || exit 1
echo done
