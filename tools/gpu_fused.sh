#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out/fused
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/fused/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/fused/pytest.log; tail -15 gpurun_out/fused/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/fused/bench.json 2> gpurun_out/fused/bench.err && cat gpurun_out/fused/bench.json && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/fused/prof -o prof --output-format csv -- python bench.py --steps 4 --warmup 2 > gpurun_out/fused/bench_prof.json 2> gpurun_out/fused/bench_prof.err
echo "done rc=$?"
