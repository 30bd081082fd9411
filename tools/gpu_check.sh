#!/bin/bash
# validation pass: kernel numerics, smoke, attention microbench, headline bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
O=gpurun_out/${OUT:-check}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log
[ $rc -eq 0 ] || exit 4
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || exit 5
tail -1 $O/smoke.log
timeout -k 10 300 python tools/attn_bench.py > $O/attn.jsonl 2> $O/attn.err || exit 6
cat $O/attn.jsonl
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 7
cat $O/bench.json
echo "all done"
