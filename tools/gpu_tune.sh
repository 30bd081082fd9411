#!/bin/bash
# TunableOp tuning pass over the headline bench shapes (incl. split-K batched wgrad GEMMs)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
O=gpurun_out/tune
mkdir -p $O
export PYTHONUNBUFFERED=1
APEX_TUNABLEOP_TUNE=1 PYTORCH_TUNABLEOP_VERBOSE=1 PYTORCH_TUNABLEOP_FILENAME=$PWD/$O/tunableop_results%d.csv \
timeout -k 10 900 python bench.py --steps 2 --warmup 2 > $O/bench_tune.json 2> $O/bench_tune.err; rc=$?; cat $O/bench_tune.json
[ $rc -eq 0 ] || exit 4
PYTORCH_TUNABLEOP_FILENAME=$PWD/$O/tunableop_results%d.csv timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json
[ $rc -eq 0 ] || exit 5
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/bench_old.json 2> $O/bench_old.err; rc=$?; cat $O/bench_old.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 -L > $O/counters_avail.txt 2>&1
echo "all done"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_gpt2 -o prof --output-format csv -- python benchmarks/gpt2.py --steps 3 --warmup 1 > $O/gpt2_prof.json 2> $O/gpt2_prof.err || exit 9
echo "gpt2 prof done"
