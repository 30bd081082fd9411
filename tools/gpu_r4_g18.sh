#!/bin/bash
# round 4: validation — full GPU suite, smoke(), bench (bf16 + fp32 pass)
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -q -m gpu -x --timeout 120 --timeout-method thread tests/ > $O/g18_gpu_suite.log 2>&1 || exit 1
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/g18_smoke.log 2>&1 || exit 1
$T 600 python bench.py --steps 10 --warmup 4 > $O/g18_bench.json 2> $O/g18_bench.err || exit 1
echo done
