#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
O=gpurun_out/attn4
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -x > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 300 python tools/attn_bench.py > $O/attn.jsonl 2> $O/attn.err; rc=$?; cat $O/attn.jsonl
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json
[ $rc -eq 0 ] || exit 5
APEX_TUNABLEOP_TUNE=1 PYTORCH_TUNABLEOP_FILENAME=$PWD/$O/tune_gpt2_%d.csv timeout -k 10 600 python benchmarks/gpt2.py --steps 2 --warmup 2 > $O/gpt2_tune.json 2> $O/gpt2_tune.err; rc=$?; cat $O/gpt2_tune.json
[ $rc -eq 0 ] || exit 6
APEX_TUNABLEOP_TUNE=1 PYTORCH_TUNABLEOP_FILENAME=$PWD/$O/tune_meg_%d.csv timeout -k 10 600 python benchmarks/megatron_gpt.py --steps 2 --warmup 1 --global-batch 8 > $O/meg_tune.json 2> $O/meg_tune.err; rc=$?; cat $O/meg_tune.json
[ $rc -eq 0 ] || exit 7
timeout -k 10 300 python benchmarks/gpt2.py --steps 5 --warmup 2 > $O/gpt2.json 2> $O/gpt2.err; rc=$?; cat $O/gpt2.json
echo "all done"
