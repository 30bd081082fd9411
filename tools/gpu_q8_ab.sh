#!/bin/bash
# fp8 producer-code change: attention / fp8 GPU tests, then a same-box A/B (previous build vs the
# tree's) of tools/f8_producer_bench.py and of bench.py --fp8
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-q8ab}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py tests/test_attention_gpu.py tests/test_attention_ext_gpu.py \
  tests/test_attention_bias_grad_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 3; }
tail -2 $O/pytest.log
bash tools/gpu_so_ab.sh ${OUT:-q8ab}/prod 2 "python tools/f8_producer_bench.py"
bash tools/gpu_so_ab.sh ${OUT:-q8ab}/bench 1 "python bench.py --steps 10 --warmup 3 --fp8"
echo done
