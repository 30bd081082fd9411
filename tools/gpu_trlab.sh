#!/bin/bash
# Weight-gradient (transposed-read) GEMM lab: labbin/trlab (tools/gemmlab/tr_lab.hip) at the
# BERT-Large weight shapes, M = 98304 tokens. Env: OUT (gpurun_out subdir), SHAPES (override,
# ';'-separated "P Q R splits").
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-trlab}
mkdir -p $O
SH=${SHAPES:-"4096 1024 98304 4;1024 4096 98304 4;3072 1024 98304 4;3072 1024 98304 16;1024 1024 98304 16"}
IFS=';' read -ra A <<< "$SH"
for s in "${A[@]}"; do
  timeout -k 5 120 labbin/trlab $s 3 5 >> $O/trlab.jsonl 2>> $O/trlab.err || { echo "FAILED: $s"; tail -5 $O/trlab.err; exit 3; }
done
cat $O/trlab.jsonl
