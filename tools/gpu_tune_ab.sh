#!/bin/bash
# Same-box A/B of two TunableOp result files on the GPT-2 and Megatron benches:
# new = tuning/ (in-tree), old = $OLD_DIR/tunableop_results0.csv
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-tuneab}
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then X="PYTORCH_TUNABLEOP_FILENAME=$PWD/$OLD_DIR/tunableop_results%d.csv"; else X="APEX_AB=new"; fi
    for B in ${BENCHES:-gpt2 megatron_gpt}; do
      env $X timeout -k 10 400 python benchmarks/$B.py > $O/${B}_$v$r.json 2> $O/${B}_$v$r.err || { tail -5 $O/${B}_$v$r.err; exit 5; }
      echo "$v $B $(python -c "import json;d=json.load(open('$O/${B}_$v$r.json'));print(d['value'], d['ms_per_step'], d['tunableop']['results_loaded'])")"
    done
  done
done
echo "all done"
