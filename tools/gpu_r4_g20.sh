#!/bin/bash
# round 4: same-box A/B of the GELU epilogue math (folded constants) on the FFN1 GEMM: lab binary
# built from the previous commit vs the current tree, interleaved
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
: > $O/g20_gelu_ab.jsonl
for r in 1 2 3; do
  for b in gemmlab_prev gemmlab; do
    timeout -k 10 120 labbin/$b 98304 4096 1024 8 3 10 | sed "s/\"variant\": \"w8\"/\"variant\": \"w8_$b\"/" | grep "w8_$b" >> $O/g20_gelu_ab.jsonl || exit 1
  done
done
cat $O/g20_gelu_ab.jsonl
