#!/bin/bash
# round 4: GELU epilogue math with folded constants — GEMM / fp8 / MLP tests, lab timing, bench
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
T="timeout -k 10"
PT="python -u -m pytest -q -x --timeout 120 --timeout-method thread"
$T 400 $PT tests/test_gemm_gpu.py tests/test_fp8_gpu.py tests/test_fused_ops_gpu.py > $O/g19_tests.log 2>&1 || exit 1
: > $O/g19_gemmlab.jsonl
for shp in "98304 4096 1024 8"; do
  $T 120 labbin/gemmlab $shp 5 10 >> $O/g19_gemmlab.jsonl 2>> $O/g19_gemmlab.err || exit 1
done
$T 600 python bench.py --steps 10 --warmup 4 --no-fp32 > $O/g19_bench.json 2> $O/g19_bench.err || exit 1
echo done
