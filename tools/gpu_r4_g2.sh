#!/bin/bash
# round 4: attention dropout stream RNG + SHORT/DB dropout knobs; fp32 dense path; bench + step profile
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
T="timeout -k 10"
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
$T 400 $PT tests/test_attention_gpu.py tests/test_attention_ext_gpu.py tests/test_attention_fp32_gpu.py tests/test_chunked_attention.py > $O/g2_attn_tests.log 2>&1 || exit 1
APEX_ATTN_FWD_SHORT_DROP=1 APEX_ATTN_FWD_DB_DROP=1 $T 400 $PT tests/test_attention_gpu.py tests/test_attention_ext_gpu.py > $O/g2_attn_tests_knobs.log 2>&1 || exit 1
for v in "base" "APEX_ATTN_FWD_SHORT_DROP=1" "APEX_ATTN_FWD_DB_DROP=1" "base2"; do
  for sh in bert768 gpt2; do
    env ${v/base*/X=1} $T 120 python tools/attn_bench.py --only $sh 2>/dev/null | sed "s/^/{\"variant\": \"$v\", \"r\": /; s/$/}/" >> $O/g2_attn_ab.jsonl || exit 1
  done
done
$T 400 python bench.py --steps 10 --warmup 4 > $O/g2_bench.json 2> $O/g2_bench.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$T 400 rocprofv3 --kernel-trace --stats -d $O/g2prof -o prof --output-format csv -- python bench.py --steps 4 --warmup 3 --no-fp32 > $O/g2_prof_bench.json 2> $O/g2_prof.err || exit 1
f=$(find $O/g2prof -name "*kernel_trace.csv" | head -1)
python tools/profstep.py "$f" 3 45 > $O/g2_step_kernels.txt
rm -f "$f"
echo done
