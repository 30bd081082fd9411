#!/bin/bash
# round 4: BERT weight-gradient GEMMs — production split-K batched GEMM vs one TunableOp-tuned GEMM
set -o pipefail
O=gpurun_out/r4; mkdir -p $O/wgrad_tune
( while true; do sleep 30; echo "tick $(date +%s)"; done ) &
TICK=$!
timeout -k 10 900 python tools/wgrad_tune_bench.py --out $PWD/$O/wgrad_tune/tunableop_results%d.csv > $O/g17_wgrad.jsonl 2> $O/g17_wgrad.err
rc=$?
kill $TICK
cat $O/g17_wgrad.jsonl
exit $rc
