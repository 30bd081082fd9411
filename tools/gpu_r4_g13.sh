#!/bin/bash
# round 4: GEMM lab — w8p (per-wave software-pipelined fragment reads, one barrier per K-tile) vs the
# ping-pong w8, with and without the MFMA/ds_read interleave hints, full kernels and main loops
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
: > $O/g13_gemmlab.jsonl
for shp in "8192 8192 8192 0" "98304 1024 1024 0" "98304 1024 4096 4" "98304 4096 1024 8"; do
  LAB_NOEPI=1 timeout -k 10 120 labbin/gemmlab $shp 5 10 >> $O/g13_gemmlab.jsonl 2>> $O/g13_gemmlab.err || { echo "lab failed: $shp"; exit 1; }
  timeout -k 10 120 labbin/gemmlab_nosched $shp 3 10 | sed 's/"w8p"/"w8p_nosched"/' >> $O/g13_gemmlab.jsonl 2>> $O/g13_gemmlab.err || { echo "lab nosched failed: $shp"; exit 1; }
done
echo done
