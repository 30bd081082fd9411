#!/bin/bash
# fp32 main_grad on the transposed-read MFMA kernel (gemm_tt_acc): GPU tests, per-shape A/B at the
# Megatron wgrad shapes, and the Megatron bench with APEX_MAIN_GRAD_GEMM=auto vs lib vs bf16 grads
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-mg}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_main_grad_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/main_grad_ab.py 8192 2560 > $O/ab.jsonl 2> $O/ab.err || { tail -20 $O/ab.err; exit 4; }
cat $O/ab.jsonl
timeout -k 10 400 python benchmarks/megatron_gpt.py > $O/meg_auto.json 2> $O/meg_auto.err || { tail -20 $O/meg_auto.err; exit 5; }
APEX_MAIN_GRAD_GEMM=lib timeout -k 10 400 python benchmarks/megatron_gpt.py > $O/meg_lib.json 2> $O/meg_lib.err || { tail -20 $O/meg_lib.err; exit 6; }
timeout -k 10 400 python benchmarks/megatron_gpt.py --bf16-grad-accum > $O/meg_bf16.json 2> $O/meg_bf16.err || { tail -20 $O/meg_bf16.err; exit 7; }
cut -c1-220 $O/meg_auto.json $O/meg_lib.json $O/meg_bf16.json
echo "all done"
