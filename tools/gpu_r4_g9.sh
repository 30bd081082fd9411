#!/bin/bash
# round 4: GEMM lab — 32x32x16-fragment variant of the 8-wave ping-pong kernel (w8m32) vs the
# 16x16x32 production kernel (w8), full kernels and main loops alone (noepi), BERT shapes + 8192^3
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
: > $O/g9_gemmlab.jsonl
for shp in "8192 8192 8192 0" "98304 1024 1024 0" "98304 3072 1024 0" "98304 1024 4096 4" "98304 4096 1024 8" "98304 4096 1024 10"; do
  LAB_NOEPI=1 timeout -k 10 120 labbin/gemmlab $shp 5 10 >> $O/g9_gemmlab.jsonl 2>> $O/g9_gemmlab.err || { echo "lab failed: $shp"; exit 1; }
done
APEX_GEMM_M32=all timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > $O/g9_gemm_m32_tests.log 2>&1 || { echo "m32 gemm tests failed"; exit 1; }
timeout -k 10 180 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tools/rccl_two_ranks_one_gpu.py > $O/g9_rccl_two_ranks.json 2> $O/g9_rccl_two_ranks.err || echo "rccl two-rank run failed (see err)"
echo done
