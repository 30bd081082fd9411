#!/bin/bash
# round 4: ring-attention emulation kernel breakdown (rocprofv3 stats) + the w8p lab variant with
# buffer-resource staging
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_context_parallel_gpu.py > $O/g14_cp_tests.log 2>&1 || { echo "cp tests failed"; exit 1; }
timeout -k 10 200 python tools/cp_emul_bench.py --S 16384 > $O/g14_cp_emul16k.jsonl 2> $O/g14_cp_emul16k.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/g14prof -o cp --output-format csv -- python tools/cp_emul_bench.py > $O/g14_cp_emul.jsonl 2> $O/g14_cp_emul.err || { echo "cp prof failed"; exit 1; }
f=$(find $O/g14prof -name "*kernel_stats.csv" | head -1)
cp $f $O/g14_cp_kernel_stats.csv
rm -rf $O/g14prof
: > $O/g14_gemmlab.jsonl
for shp in "8192 8192 8192 0" "98304 4096 1024 8"; do
  LAB_NOEPI=1 timeout -k 10 120 labbin/gemmlab $shp 3 10 >> $O/g14_gemmlab.jsonl 2>> $O/g14_gemmlab.err || { echo "lab failed: $shp"; exit 1; }
done
echo done
