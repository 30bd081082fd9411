#!/bin/bash
# round 4: balanced GEMM main loop + TR weight gradients for the FFN shapes: GEMM/fp8/fused tests,
# the weight-gradient A/B, the lab, then the headline bench
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_fp8_gpu.py tests/test_fused_ops_gpu.py tests/test_main_grad_gpu.py tests/test_gpt_fused_gpu.py tests/test_ddp_race_gpu.py > $O/g25_tests.txt 2>&1 || { tail -30 $O/g25_tests.txt; exit 1; }
tail -2 $O/g25_tests.txt
timeout -k 10 300 python tools/wgrad_tt_bench.py > $O/g25_wgrad_tt.jsonl || exit 2
cat $O/g25_wgrad_tt.jsonl
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/g25_bench.json 2> $O/g25_bench.err || { tail $O/g25_bench.err; exit 3; }
python -c "import json;d=json.load(open('$O/g25_bench.json'));print(d['value'],d['ms_per_step'],d.get('extra',{}).get('gpu',d.get('gpu')))" || tail -3 $O/g25_bench.json
