#!/bin/bash
# Weight gradients without split-K (APEX_WGRAD_SPLITK=0: one library GEMM per dW, TunableOp-tuned —
# hipBLASLt's stream-K kernels split the long contraction internally) vs the split-K batched path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-wgt}
mkdir -p $O/tune
export PYTHONUNBUFFERED=1
cp tuning/tunableop_results0.csv $O/tune/tunableop_results0.csv
( while true; do sleep 30; echo "tick $(wc -l < $O/tune/tunableop_results0.csv)"; done ) &
TICK=$!
APEX_WGRAD_SPLITK=0 PYTORCH_TUNABLEOP_FILENAME=$PWD/$O/tune/tunableop_results%d.csv APEX_TUNABLEOP_TUNE=1 \
  timeout -k 10 900 python bench.py --steps 2 --warmup 1 --no-fp32 > $O/tune.json 2> $O/tune.err || { kill $TICK; tail -5 $O/tune.err; exit 3; }
kill $TICK
grep -v Validator $O/tune/tunableop_results0.csv | grep "_98304_" | grep "^GemmTunableOp_BFloat16_NT" || true
for r in 1 2; do
  APEX_WGRAD_SPLITK=0 PYTORCH_TUNABLEOP_FILENAME=$PWD/$O/tune/tunableop_results%d.csv timeout -k 10 400 python bench.py --no-fp32 > $O/nosplit$r.json 2> $O/nosplit$r.err || exit 4
  echo "nosplit tuned $(python -c "import json;d=json.load(open('$O/nosplit$r.json'));print(d['value'], d['ms_per_step'])")"
  timeout -k 10 400 python bench.py --no-fp32 > $O/split$r.json 2> $O/split$r.err || exit 5
  echo "split-K      $(python -c "import json;d=json.load(open('$O/split$r.json'));print(d['value'], d['ms_per_step'])")"
done
echo "all done"
