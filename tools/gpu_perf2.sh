#!/bin/bash
# attention bwd pipelining + lds barriers; tuned-GEMM bench; GEMM split-K microbench; profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
O=gpurun_out/perf2
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_attention_gpu.py tests/test_optim_mixed_gpu.py tests/test_multihead_attn.py tests/test_fused_ops_gpu.py -m gpu -q -rf > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest.log; tail -5 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json
[ $rc -eq 0 ] || exit 4
APEX_TUNABLEOP=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_untuned.json 2> $O/bench_untuned.err; rc=$?; cat $O/bench_untuned.json
[ $rc -eq 0 ] || exit 5
timeout -k 10 300 python tools/gemm_bench.py > $O/gemm.jsonl 2> $O/gemm.err; rc=$?; cat $O/gemm.jsonl
[ $rc -eq 0 ] || exit 6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- python bench.py --steps 4 --warmup 2 > $O/bench_prof.json 2> $O/bench_prof.err || exit 9
echo "all done"
