#!/bin/bash
# round 4: ring-step key split across two streams (CP tests + emulation with and without)
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_context_parallel_gpu.py > $O/g15_cp_tests.log 2>&1 || { echo "cp tests failed"; exit 1; }
: > $O/g15_cp_emul.jsonl
for S in 8192 16384; do
  $T 200 python tools/cp_emul_bench.py --S $S >> $O/g15_cp_emul.jsonl 2>> $O/g15_cp_emul.err || exit 1
  APEX_CP_KV_SPLIT=0 $T 200 python tools/cp_emul_bench.py --S $S >> $O/g15_cp_emul.jsonl 2>> $O/g15_cp_emul.err || exit 1
done
echo done
