#!/bin/bash
# round 4 final validation (balanced GEMM loop, TR FFN weight gradients) — full GPU suite, smoke(), bench (bf16 + fp32 pass)
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -q -m gpu -x --timeout 120 --timeout-method thread tests/ > $O/g30_gpu_suite.log 2>&1 || exit 1
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/g30_smoke.log 2>&1 || exit 1
$T 600 python bench.py --steps 10 --warmup 4 > $O/g30_bench.json 2> $O/g30_bench.err || exit 1
echo done
tail -2 $O/g30_gpu_suite.log; tail -2 $O/g30_smoke.log; python -c "import json;d=json.load(open(\"$O/g30_bench.json\"));print(d[\"value\"],d[\"ms_per_step\"],d.get(\"speedup_vs_fp32\"),d[\"gpu\"][\"timed\"][\"sclk_mhz\"])"
