#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out/attn
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -m pytest tests/test_attention_gpu.py -q -rf -x > gpurun_out/attn/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/attn/pytest.log; tail -15 gpurun_out/attn/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/attn/bench.json 2> gpurun_out/attn/bench.err && cat gpurun_out/attn/bench.json && \
APEX_ATTN_BACKEND=sdpa timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/attn/bench_sdpa.json 2> gpurun_out/attn/bench_sdpa.err && cat gpurun_out/attn/bench_sdpa.json && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/attn/prof -o prof --output-format csv -- python bench.py --steps 4 --warmup 2 > gpurun_out/attn/bench_prof.json 2> gpurun_out/attn/bench_prof.err
echo "done rc=$?"
