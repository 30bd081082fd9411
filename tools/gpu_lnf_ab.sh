#!/bin/bash
# LayerNorm forward load-phase change: LN / fp8 GPU tests, then previous build vs this one (bandwidth probe, bench)
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lnf
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py tests/test_post_ln_mem_gpu.py tests/test_fused_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lnf/pytest.log 2>&1 || { tail -30 gpurun_out/lnf/pytest.log; exit 3; }
tail -1 gpurun_out/lnf/pytest.log
bash tools/gpu_so_ab.sh lnf/probe 2 "python tools/bdaln_bw_probe.py"
bash tools/gpu_so_ab.sh lnf/bench 2 "python bench.py --steps 20 --warmup 5 --no-fp32"
