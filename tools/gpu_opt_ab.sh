#!/bin/bash
# Same-box A/B of the optimizer streams: labbin/_C_old.so (the build before the change) against
# the tree's build, interleaved twice, tools/bw_kernels.py --ops lamb,adam. Then the optimizer
# GPU tests on the new build.
set -euo pipefail
OUT=gpurun_out/${1:-opt_ab}
mkdir -p "$OUT"
SO=apex/_C.cpython-310-x86_64-linux-gnu.so
cp "$SO" labbin/_C_new.so
for r in 1 2; do
  for b in old new; do
    cp "labbin/_C_$b.so" "$SO"
    timeout -k 10 300 python -u tools/bw_kernels.py --ops lamb,adam --iters 10 > "$OUT/${b}_$r.jsonl"
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "lamb or adam or sgd or optim" > "$OUT/tests.txt" 2>&1
