#!/bin/bash
# TunableOp: add the GPT-2 1.5B and Megatron GPT GEMM shapes to the committed BERT selections, then a
# same-box A/B of both benches with the old and the merged file. Output: gpurun_out/$OUT/tune/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-tunem}
mkdir -p $O/tune
export PYTHONUNBUFFERED=1
cp tuning/tunableop_results0.csv $O/tune/tunableop_results0.csv
T="PYTORCH_TUNABLEOP_FILENAME=$PWD/$O/tune/tunableop_results%d.csv APEX_TUNABLEOP_TUNE=1"
env $T timeout -k 10 500 python benchmarks/gpt2.py --steps 2 --warmup 1 > $O/tune_gpt2.json 2> $O/tune_gpt2.err || { tail -5 $O/tune_gpt2.err; exit 3; }
env $T timeout -k 10 500 python benchmarks/megatron_gpt.py --steps 2 --warmup 1 --global-batch 8 > $O/tune_meg.json 2> $O/tune_meg.err || { tail -5 $O/tune_meg.err; exit 4; }
wc -l tuning/tunableop_results0.csv $O/tune/tunableop_results0.csv
for r in 1 2; do
  for v in old new; do
    if [ $v = new ]; then X="PYTORCH_TUNABLEOP_FILENAME=$PWD/$O/tune/tunableop_results%d.csv"; else X="APEX_AB=old"; fi
    for B in gpt2 megatron_gpt; do
      env $X timeout -k 10 400 python benchmarks/$B.py > $O/${B}_$v$r.json 2> $O/${B}_$v$r.err || { tail -5 $O/${B}_$v$r.err; exit 5; }
      echo "$v $B $(python -c "import json;d=json.load(open('$O/${B}_$v$r.json'));print(d['value'], d['ms_per_step'], d['tunableop']['results_loaded'])")"
    done
  done
done
echo "all done"
