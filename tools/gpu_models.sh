#!/bin/bash
# GPU session: full gpu test tier, headline bench (bf16 + fp32), model-zoo benches, profiles.
# Stops at the first crash / timeout (rc not in {0,1}); test failures (rc 1) do not stop it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
O=gpurun_out/models
mkdir -p $O
export PYTHONUNBUFFERED=1
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 700 python -m pytest tests -m gpu -q -rf -x > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest.log; tail -12 $O/pytest.log
ok $rc || exit 3
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json
[ $rc -eq 0 ] || exit 4
timeout -k 10 300 python bench.py --fp32 --steps 5 --warmup 2 > $O/bench_fp32.json 2> $O/bench_fp32.err; rc=$?; cat $O/bench_fp32.json
[ $rc -eq 0 ] || exit 5
timeout -k 10 300 python benchmarks/resnet50.py --steps 10 --warmup 3 > $O/resnet50.json 2> $O/resnet50.err; rc=$?; cat $O/resnet50.json
[ $rc -eq 0 ] || exit 6
timeout -k 10 300 python benchmarks/gpt2.py --steps 5 --warmup 2 > $O/gpt2.json 2> $O/gpt2.err; rc=$?; cat $O/gpt2.json
[ $rc -eq 0 ] || exit 7
timeout -k 10 300 python benchmarks/megatron_gpt.py --steps 3 --warmup 1 --global-batch 8 > $O/megatron.json 2> $O/megatron.err; rc=$?; cat $O/megatron.json
[ $rc -eq 0 ] || exit 8
echo "all done"
