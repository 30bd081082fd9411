#!/bin/bash
# attention bwd occupancy change + mixed-dtype optimizers; model benches; TunableOp GEMM tuning trial
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
O=gpurun_out/perf1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_attention_gpu.py tests/test_optim_mixed_gpu.py tests/test_utils.py tests/test_multihead_attn.py -m gpu -q -rf > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest.log; tail -8 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json
[ $rc -eq 0 ] || exit 4
timeout -k 10 300 python benchmarks/resnet50.py --steps 10 --warmup 3 > $O/resnet50.json 2> $O/resnet50.err; rc=$?; cat $O/resnet50.json; tail -2 $O/resnet50.err
[ $rc -eq 0 ] || exit 6
timeout -k 10 300 python benchmarks/gpt2.py --steps 5 --warmup 2 > $O/gpt2.json 2> $O/gpt2.err; rc=$?; cat $O/gpt2.json; tail -2 $O/gpt2.err
[ $rc -eq 0 ] || exit 7
timeout -k 10 300 python benchmarks/megatron_gpt.py --steps 3 --warmup 1 --global-batch 8 > $O/megatron.json 2> $O/megatron.err; rc=$?; cat $O/megatron.json; tail -2 $O/megatron.err
[ $rc -eq 0 ] || exit 8
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=8 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=2 \
PYTORCH_TUNABLEOP_FILENAME=$O/tunableop_results%d.csv \
timeout -k 10 900 python bench.py --steps 3 --warmup 2 > $O/bench_tune.json 2> $O/bench_tune.err; rc=$?; cat $O/bench_tune.json
[ $rc -eq 0 ] || exit 9
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop_results%d.csv \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_tuned.json 2> $O/bench_tuned.err; rc=$?; cat $O/bench_tuned.json
echo "all done rc=$rc"
