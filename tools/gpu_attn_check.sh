#!/bin/bash
# attention GPU tests + microbenchmark (+ optional model bench given in $BENCH)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-attn}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_multihead_attn.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/attn_bench.py > $O/attn_bench.jsonl 2> $O/attn_bench.err || { tail -20 $O/attn_bench.err; exit 4; }
cat $O/attn_bench.jsonl
if [ -n "$BENCH" ]; then
  timeout -k 10 400 $BENCH > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 5; }
  cat $O/bench.json
fi
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  for CASE in "bert fwd 0.1" "bert bwd 0.1" "gpt2 fwd 0.1" "gpt2 bwd 0.1"; do set -- $CASE
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_$1_$2 -o p --output-format csv -- python tools/attn_one.py $1 $2 $3 10 > $O/prof_$1_$2.log 2>&1 || { echo "prof $CASE failed"; exit 6; }
  done
fi
echo "all done"
