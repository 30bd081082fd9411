#!/bin/bash
# GEMM tile-order sweep: labbin/gemmlab_g{4,8,16,32} (tools/gemmlab/lab.hip built with
# -DAPEX_G_GROUP_M=G) on the BERT shapes at M = 98304, binaries interleaved per shape; every JSON line
# gains "group_m". Env: OUT (gpurun_out subdir), SHAPES (override, ';'-separated), GS (group sizes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-groupm}
mkdir -p $O
SH=${SHAPES:-"98304 3072 1024 1;98304 1024 1024 0;98304 4096 1024 8;98304 1024 4096 4;98304 4096 1024 10;8192 8192 8192 0 3 5"}
GS=${GS:-"8 4 16 32"}
IFS=';' read -ra A <<< "$SH"
for s in "${A[@]}"; do
  for g in $GS; do
    timeout -k 5 90 labbin/gemmlab_g$g $s 2>> $O/lab.err | sed "s/^{/{\"group_m\": $g, /" >> $O/lab.jsonl || { echo "FAILED: g$g $s"; tail -5 $O/lab.err; exit 3; }
  done
done
cat $O/lab.jsonl
