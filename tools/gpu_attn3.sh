#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
O=gpurun_out/attn3
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_attention_gpu.py tests/test_multihead_attn.py tests/test_fused_ops_gpu.py -m gpu -q -rf > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 300 python tools/attn_bench.py > $O/attn.jsonl 2> $O/attn.err; rc=$?; cat $O/attn.jsonl
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json
[ $rc -eq 0 ] || exit 5
echo "all done"
