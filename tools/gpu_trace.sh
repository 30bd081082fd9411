#!/bin/bash
# GEMM timeline trace (labbin/gemmlab built from tools/gemmlab/lab.hip, LAB_TRACE=1): per-workgroup
# main-loop / epilogue / dispatch-gap durations and epilogue concurrency at the BERT shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-trace}
mkdir -p $O
L=labbin/${LAB:-gemmlab}
export LAB_TRACE=1
for s in "98304 1024 1024 0" "98304 3072 1024 1" "98304 4096 1024 8" "98304 1024 4096 4" "98304 4096 1024 10" "98304 1024 3072 4"; do
  timeout -k 5 60 $L $s 3 5 >> $O/trace.jsonl 2>> $O/trace.err || { echo "FAILED: $s"; tail -5 $O/trace.err; exit 3; }
done
cat $O/trace.jsonl
