#!/bin/bash
# Experiment: bf16 split-K slabs (TunableOp-tuned batched GEMM) vs fp32 slabs, BERT b768.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-wslab}
mkdir -p $O/tune
export PYTHONUNBUFFERED=1
cp tuning/tunableop_results0.csv $O/tune/tunableop_results0.csv
( while true; do sleep 30; echo "tick $(wc -l < $O/tune/tunableop_results0.csv)"; done ) &
TICK=$!
APEX_WGRAD_SLAB=bf16 PYTORCH_TUNABLEOP_FILENAME=$PWD/$O/tune/tunableop_results%d.csv APEX_TUNABLEOP_TUNE=1 \
  timeout -k 10 900 python bench.py --steps 2 --warmup 1 --no-fp32 > $O/tune.json 2> $O/tune.err || { kill $TICK; tail -5 $O/tune.err; exit 3; }
kill $TICK
grep -i "batched" $O/tune/tunableop_results0.csv || true
for r in 1 2; do
  APEX_WGRAD_SLAB=bf16 PYTORCH_TUNABLEOP_FILENAME=$PWD/$O/tune/tunableop_results%d.csv timeout -k 10 400 python bench.py --no-fp32 > $O/bf16_$r.json 2> $O/bf16_$r.err || exit 4
  echo "bf16 slabs $(python -c "import json;d=json.load(open('$O/bf16_$r.json'));print(d['value'], d['ms_per_step'])")"
  timeout -k 10 400 python bench.py --no-fp32 > $O/fp32_$r.json 2> $O/fp32_$r.err || exit 5
  echo "fp32 slabs $(python -c "import json;d=json.load(open('$O/fp32_$r.json'));print(d['value'], d['ms_per_step'])")"
done
echo "all done"
