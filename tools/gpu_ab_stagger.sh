#!/bin/bash
# A/B of the per-epilogue GEMM first-round stagger (APEX_GEMM_STAGGER) on the headline step,
# interleaved on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
O=gpurun_out/${OUT:-ab_stagger}
mkdir -p $O
for rep in 1 2; do
  for cfg in "none" "8:1,10:1" "8:2,10:2" "8:2,10:2,4:1"; do
    tag=$(echo "$cfg" | tr ':,' '_-')
    if [ "$cfg" = "none" ]; then env_cfg=""; else env_cfg="$cfg"; fi
    APEX_GEMM_STAGGER="$env_cfg" timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-fp32 > $O/b_${tag}_$rep.json 2> $O/b_${tag}_$rep.err || exit $?
    python -c "import json,sys; d=json.loads(open('$O/b_${tag}_$rep.json').read().strip().splitlines()[-1]); print('$cfg', $rep, d['value'], d['ms_per_step'], d['gpu']['timed']['sclk_mhz']['mean'])"
  done
done
