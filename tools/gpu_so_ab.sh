#!/bin/bash
# Same-box A/B of two builds of the extension: $PREV (default labbin/_C_prev.so, via APEX_EXT_SO) against the tree's
# build, interleaved. Usage: gpu_so_ab.sh OUT ROUNDS "cmd args" (cmd's stdout -> OUT/{prev,new}_r.out)
set -euo pipefail
OUT=gpurun_out/${1:?out}
ROUNDS=${2:-2}
CMD=${3:?command}
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  APEX_EXT_SO=${PREV:-labbin/_C_prev.so} timeout -k 10 400 $CMD > "$OUT/prev_$r.out" 2> "$OUT/prev_$r.err"
  timeout -k 10 400 $CMD > "$OUT/new_$r.out" 2> "$OUT/new_$r.err"
done
