#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
O=gpurun_out/perf3
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_fused_ops_gpu.py tests/test_bert_cpu.py -m gpu -q -rf > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest.log; tail -5 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json
[ $rc -eq 0 ] || exit 4
APEX_WGRAD_SPLITK=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_nosplit.json 2> $O/bench_nosplit.err; rc=$?; cat $O/bench_nosplit.json
[ $rc -eq 0 ] || exit 5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- python bench.py --steps 4 --warmup 2 > $O/bench_prof.json 2> $O/bench_prof.err || exit 9
echo "all done"
