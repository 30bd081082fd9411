#!/bin/bash
# fp8 producer-side quantisation: fp8 GPU tests, then BERT-Large bf16 + fp8 passes with the LN
# kernels writing the codes (A) vs standalone quantise passes (B, APEX_FP8_PRODUCER=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-fp8p}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py tests/test_fused_ops_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
for v in A B; do
  E=1; [ $v = B ] && E=0
  APEX_FP8_PRODUCER=$E timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-fp32 --fp8 --fp8-steps 10 > $O/b_$v.json 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 4; }
  echo "$v $(python -c "import json;d=json.load(open('$O/b_$v.json'));print(d['value'], d['ms_per_step'], d['extra'].get('fp8'))")"
done
echo "all done"
