#!/bin/bash
# rocprofv3 kernel trace of the headline step (b768) + per-shape GEMM policy table at M = 98304
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-prof_r2}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/bert -o prof --output-format csv -- python bench.py --steps 4 --warmup 3 --no-fp32 > $O/bert.json 2> $O/bert.err || exit $?
f=$(find $O/bert -name "*kernel_trace.csv" | head -1)
python tools/profstep.py "$f" 3 45 > $O/bert_steps.txt && cat $O/bert_steps.txt | head -50
if [ -n "$POLICY" ]; then
  PB_M=98304 timeout -k 10 300 python tools/gemm_policy_bench.py > $O/policy.jsonl 2> $O/policy.err || exit $?
  cat $O/policy.jsonl
fi
