#!/bin/bash
# round 4: balanced main loop (mainloop_bal) vs production, TR (weight gradient) and NT shapes
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
: > $O/g24_trlab.jsonl; : > $O/g24_ntlab.jsonl
for sh in "3072 1024" "1024 1024" "4096 1024" "1024 4096"; do
  for s in 4 8 16; do
    timeout -k 10 60 labbin/trlab $sh 98304 $s 3 5 >> $O/g24_trlab.jsonl || { echo "trlab $sh $s failed"; exit 2; }
  done
done
for c in "8192 8192 8192 0" "98304 1024 1024 0" "98304 3072 1024 1" "98304 4096 1024 8" "98304 1024 4096 4" "98304 1024 4096 10"; do
  timeout -k 10 60 labbin/gemmlab $c 5 10 >> $O/g24_ntlab.jsonl || { echo "gemmlab $c failed"; exit 3; }
done
cat $O/g24_trlab.jsonl | grep -v nodsread | grep -v noglds
cat $O/g24_ntlab.jsonl
