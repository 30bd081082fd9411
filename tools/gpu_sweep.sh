#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
mkdir -p gpurun_out/sweep
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -rf -k "sgd or layer_norm" > gpurun_out/sweep/pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/sweep/pytest.log
for b in ${BATCHES:-64 128 256}; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --batch $b > gpurun_out/sweep/b$b.json 2> gpurun_out/sweep/b$b.err || { echo "bench b=$b failed"; tail -5 gpurun_out/sweep/b$b.err; break; }
  cat gpurun_out/sweep/b$b.json
done
