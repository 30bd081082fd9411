#!/bin/bash
# GPU tests, then the headline bench with the MFMA GEMM path and with the library GEMM path (A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
O=gpurun_out/${OUT:-ab}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log
[ $rc -eq 0 ] || exit 4
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || exit 5
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_mfma.json 2> $O/bench_mfma.err || exit 7
cat $O/bench_mfma.json
env ${AB_ENV:-APEX_GEMM=blas} timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_blas.json 2> $O/bench_blas.err || exit 8
cat $O/bench_blas.json
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- python bench.py --steps 5 --warmup 2 > $O/bench_prof.json 2> $O/bench_prof.err || exit 9
fi
echo "all done"
