#!/bin/bash
# GEMM lab (labbin/gemmlab, built on the CPU side): every BERT-Large GEMM shape at M = 98304
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-lab}
mkdir -p $O
L=labbin/${LAB:-gemmlab}
run() { timeout -k 5 60 $L "$@" >> $O/lab.jsonl 2>> $O/lab.err || { echo "FAILED: $*"; tail -5 $O/lab.err; exit 3; }; }
run 8192 8192 8192 0 3 5
run 98304 3072 1024 0
run 98304 1024 1024 0
run 98304 4096 1024 8
run 98304 1024 4096 0
run 98304 4096 1024 10
run 98304 1024 4096 4
run 98304 1024 3072 4
cat $O/lab.jsonl
