#!/bin/bash
# Same-box A/B of routing single plain-product weight shapes to the own persistent kernel
# (APEX_GEMM_VOCAB_TABLE entries) in the BERT step, interleaved
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-plaintab}
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for t in "30528x1024" "30528x1024,3072x1024" "30528x1024,1024x1024" "30528x1024,1024x4096"; do
    n=$(echo $t | tr ',' '_')
    APEX_GEMM_VOCAB_TABLE=$t timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-fp32 --no-fp8 > $O/${n}_$r.out 2> $O/${n}_$r.err || exit 3
    python -c "import json;d=json.loads(open('$O/${n}_$r.out').read().strip().splitlines()[-1]);print('$t', $r, d['value'], d['gpu']['timed']['sclk_mhz']['mean'])"
  done
done
