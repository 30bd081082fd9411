#!/bin/bash
# MFMA GEMM: numerics first, then the microbenchmark vs hipBLASLt
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
O=gpurun_out/${OUT:-gemm}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -rf --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -15 $O/pytest.log
[ $rc -eq 0 ] || exit 4
[ -n "$KSWEEP" ] && { timeout -k 10 300 python tools/gemm_ksweep.py > $O/ksweep.jsonl 2>&1 || exit 6; cat $O/ksweep.jsonl; }
[ -n "$POLICY" ] && { timeout -k 10 300 python tools/gemm_policy_bench.py > $O/policy.jsonl 2>&1 || exit 7; cat $O/policy.jsonl; }
[ -n "$NOMICRO" ] || { timeout -k 10 300 python tools/gemm_mfma_bench.py > $O/bench.jsonl 2> $O/bench.err || exit 5; }
[ -f $O/bench.jsonl ] && cat $O/bench.jsonl
echo "all done"
