#!/bin/bash
# model-zoo benches + profiles (after the first gpu_models run)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
O=gpurun_out/models2
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest.log; tail -8 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 300 python benchmarks/resnet50.py --steps 10 --warmup 3 > $O/resnet50.json 2> $O/resnet50.err; rc=$?; cat $O/resnet50.json; tail -3 $O/resnet50.err
[ $rc -eq 0 ] || exit 6
timeout -k 10 300 python benchmarks/gpt2.py --steps 5 --warmup 2 > $O/gpt2.json 2> $O/gpt2.err; rc=$?; cat $O/gpt2.json; tail -3 $O/gpt2.err
[ $rc -eq 0 ] || exit 7
timeout -k 10 300 python benchmarks/megatron_gpt.py --steps 3 --warmup 1 --global-batch 8 > $O/megatron.json 2> $O/megatron.err; rc=$?; cat $O/megatron.json; tail -3 $O/megatron.err
[ $rc -eq 0 ] || exit 8
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_resnet -o prof --output-format csv -- python benchmarks/resnet50.py --steps 4 --warmup 2 > $O/resnet_prof.json 2> $O/resnet_prof.err || exit 9
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_gpt2 -o prof --output-format csv -- python benchmarks/gpt2.py --steps 3 --warmup 1 > $O/gpt2_prof.json 2> $O/gpt2_prof.err || exit 10
echo "all done"
