#!/bin/bash
# all GPU tests, then the BASELINE model configs (headline + GPT-2 + Megatron), A/B on the GEMM policy
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
O=gpurun_out/${OUT:-models3}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log
[ $rc -eq 0 ] || exit 4
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 5
cat $O/bench.json
timeout -k 10 300 python benchmarks/gpt2.py --steps 5 --warmup 2 > $O/gpt2.json 2> $O/gpt2.err || exit 6
cat $O/gpt2.json
APEX_GEMM=blas timeout -k 10 300 python benchmarks/gpt2.py --steps 5 --warmup 2 > $O/gpt2_blas.json 2> $O/gpt2_blas.err || exit 7
cat $O/gpt2_blas.json
timeout -k 10 300 python benchmarks/megatron_gpt.py --steps 3 --warmup 1 --global-batch 8 > $O/megatron.json 2> $O/megatron.err || exit 8
cat $O/megatron.json
timeout -k 10 300 python benchmarks/resnet50.py --steps 10 --warmup 3 > $O/resnet50.json 2> $O/resnet50.err || exit 9
cat $O/resnet50.json
echo "all done"
