#!/bin/bash
# round 4: balanced loop on edge tiles (GPT-2 1.5B shapes) + GEMM tests + GPT-2 bench
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_gpt_fused_gpu.py > $O/g29_tests.txt 2>&1 || { tail -30 $O/g29_tests.txt; exit 1; }
tail -1 $O/g29_tests.txt
: > $O/g29_edge.jsonl
for c in "16384 1600 4800 4" "16384 1600 6400 4" "16384 4800 1600 1" "16384 6400 1600 8" "16384 1600 1600 0"; do
  timeout -k 10 60 labbin/gemmlab $c 5 10 >> $O/g29_edge.jsonl || { echo "lab $c failed"; exit 2; }
done
cat $O/g29_edge.jsonl
timeout -k 10 400 python benchmarks/gpt2.py > $O/g29_gpt2.json 2> $O/g29_gpt2.err || { tail $O/g29_gpt2.err; exit 3; }
tail -c 600 $O/g29_gpt2.json
