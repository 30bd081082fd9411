#!/bin/bash
# Same-box A/B of the split-major XCD remap of split-K (transposed-read) weight-gradient launches
# (APEX_GEMM_SPLIT_XCD=0: tile-major, the previous mapping): isolated bf16 / fp8 weight gradients at
# the BERT-Large shapes, then the headline bench, each interleaved twice.
set -euo pipefail
OUT=gpurun_out/${1:-split_xcd}
mkdir -p "$OUT"
for r in 1 2; do
  for x in 0 1; do
    APEX_GEMM_SPLIT_XCD=$x timeout -k 10 300 python -u tools/wgrad_tt_bench.py --splits 4,16 > "$OUT/tt_x${x}_$r.jsonl"
    APEX_GEMM_SPLIT_XCD=$x timeout -k 10 300 python -u tools/wgrad_f8_bench.py > "$OUT/f8_x${x}_$r.jsonl"
  done
done
for r in 1 2; do
  for x in 0 1; do
    APEX_GEMM_SPLIT_XCD=$x timeout -k 10 400 python bench.py > "$OUT/bench_x${x}_$r.json" 2> "$OUT/bench_x${x}_$r.err"
  done
done
