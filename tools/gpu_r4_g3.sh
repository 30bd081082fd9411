#!/bin/bash
# round 4: full GPU suite (new attention backward, CP merge kernel, conditional LN store), attention
# and CP microbenchmarks, bench
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -q -m gpu -x --timeout 120 --timeout-method thread tests/ > $O/g3_gpu_suite.log 2>&1 || exit 1
for sh in bert768 gpt2; do
  $T 120 python tools/attn_bench.py --only $sh >> $O/g3_attn.jsonl 2>/dev/null || exit 1
done
$T 200 python tools/cp_emul_bench.py > $O/g3_cp_emul.jsonl 2> $O/g3_cp_emul.err || exit 1
APEX_CP_DKV_FP32=1 $T 200 python tools/cp_emul_bench.py >> $O/g3_cp_emul.jsonl 2>> $O/g3_cp_emul.err || exit 1
$T 400 python bench.py --steps 10 --warmup 4 --no-fp32 > $O/g3_bench.json 2> $O/g3_bench.err || exit 1
echo done
