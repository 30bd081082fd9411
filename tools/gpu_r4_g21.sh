#!/bin/bash
# round 4: same-box A/B of the SHORT dropout forward at 3 vs 4 workgroups per CU (APEX_ATTN_SHORT_W4)
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
: > $O/g21_short_w4_ab.jsonl
for r in 1 2 3; do
  for w in 0 1; do
    APEX_ATTN_SHORT_W4=$w timeout -k 10 120 python tools/attn_bench.py --only bert768 2>/dev/null | grep '"p": 0.1' | grep '"fwd"' | sed "s/^{/{\"w4\": $w, /" >> $O/g21_short_w4_ab.jsonl || exit 1
  done
done
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_attention_ext_gpu.py > $O/g21_tests_default.log 2>&1 || exit 1
APEX_ATTN_SHORT_W4=1 timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_attention_ext_gpu.py > $O/g21_tests_w4.log 2>&1 || exit 1
cat $O/g21_short_w4_ab.jsonl
