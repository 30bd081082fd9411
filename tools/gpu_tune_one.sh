#!/bin/bash
# TunableOp tuning of one benchmark's GEMM shapes on top of a starting results file.
# Usage: OUT=dir START=path/to/tunableop_results0.csv BENCH="benchmarks/gpt2.py --steps 2 --warmup 1"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-tune1}
mkdir -p $O/tune
export PYTHONUNBUFFERED=1
cp ${START:-tuning/tunableop_results0.csv} $O/tune/tunableop_results0.csv
( while true; do sleep 30; echo "tick $(date +%s) $(wc -l < $O/tune/tunableop_results0.csv)"; done ) &
TICK=$!
PYTORCH_TUNABLEOP_FILENAME=$PWD/$O/tune/tunableop_results%d.csv APEX_TUNABLEOP_TUNE=1 PYTORCH_TUNABLEOP_ROCBLAS_ENABLED=${ROCBLAS:-0} \
  timeout -k 10 ${TLIM:-1000} python $BENCH > $O/tune.json 2> $O/tune.err
rc=$?
kill $TICK
wc -l $O/tune/tunableop_results0.csv
tail -3 $O/tune.err
exit $rc
