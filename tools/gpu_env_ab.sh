#!/bin/bash
# GPU tests in $TESTS, then the headline bench interleaved A (default env) / B ($B_ENV) twice
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-envab}
mkdir -p $O
export PYTHONUNBUFFERED=1
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
  tail -1 $O/pytest.log
fi
for rep in 1 2; do
  for v in A B; do
    if [ $v = B ]; then X="$B_ENV"; else X="APEX_AB=A"; fi
    env $X timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bert_${v}$rep.json 2> $O/bert_${v}$rep.err || { tail -5 $O/bert_${v}$rep.err; exit 4; }
    echo "$v bert $(python -c "import json;d=json.load(open('$O/bert_${v}$rep.json'));print(d['value'], d['ms_per_step'], d.get('peak_mem_gb'), d['gpu'].get('timed',{}).get('sclk_mhz_mean') if isinstance(d.get('gpu'),dict) else '')")"
  done
done
echo "all done"
