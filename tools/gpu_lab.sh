#!/bin/bash
# GEMM lab (labbin/gemmlab, built on the CPU side from tools/gemmlab/lab.hip): the BERT-Large GEMM
# shapes at M = 98304 (+ 8192^3); every variant interleaved in one process, outputs checked against
# the production kernel. Env: OUT (gpurun_out subdir), LAB (binary), SHAPES (override, ';'-separated),
# plus the lab's own LAB_* switches (LAB_TRACE, LAB_DBG, LAB_NOPERSIST, ...).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-lab}
mkdir -p $O
L=labbin/${LAB:-gemmlab}
SH=${SHAPES:-"8192 8192 8192 0 3 5;98304 3072 1024 1;98304 1024 1024 0;98304 4096 1024 8;98304 1024 4096 4;98304 4096 1024 10;98304 1024 3072 4;98304 1024 1024 4"}
IFS=';' read -ra A <<< "$SH"
for s in "${A[@]}"; do
  timeout -k 5 90 $L $s >> $O/lab.jsonl 2>> $O/lab.err || { echo "FAILED: $s"; tail -5 $O/lab.err; exit 3; }
done
cat $O/lab.jsonl
