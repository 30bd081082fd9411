#!/bin/bash
# first GPU validation: kernel numerics, smoke, short bench, rocprof stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && echo smoke-ok && \
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err && cat gpurun_out/bench1.json && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o prof --output-format csv -- python bench.py --steps 5 --warmup 2 > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
echo "done rc=$?"
