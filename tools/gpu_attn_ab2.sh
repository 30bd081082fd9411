#!/bin/bash
# attention kernels: GPU tests on the in-tree build (A), then A/B timing vs $SO_B interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-attnab}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_attention_ext_gpu.py tests/test_multihead_attn.py tests/test_context_parallel_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in A B; do
    if [ $v = B ]; then X="APEX_EXT_SO=$SO_B"; else X="APEX_AB=A"; fi
    for S in ${SHAPES:-bert gpt2}; do
      env $X timeout -k 10 200 python tools/attn_bench.py --only $S > $O/${S}_${v}$rep.jsonl 2> $O/${S}_${v}$rep.err || { tail -5 $O/${S}_${v}$rep.err; exit 4; }
      sed "s/^/$v$rep /" $O/${S}_${v}$rep.jsonl
    done
  done
done
echo "all done"
