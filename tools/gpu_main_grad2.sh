#!/bin/bash
# Megatron GPT: fp32 main_grad (deferred multi-tensor adds + gemm_tt_acc policy) vs bf16 .grad
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-mg2}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_main_grad_gpu.py tests/test_ddp_rccl_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
timeout -k 10 400 python benchmarks/megatron_gpt.py > $O/meg_auto.json 2> $O/meg_auto.err || { tail -20 $O/meg_auto.err; exit 5; }
timeout -k 10 400 python benchmarks/megatron_gpt.py --bf16-grad-accum > $O/meg_bf16.json 2> $O/meg_bf16.err || { tail -20 $O/meg_bf16.err; exit 7; }
cut -c1-220 $O/meg_auto.json $O/meg_bf16.json
echo "all done"
