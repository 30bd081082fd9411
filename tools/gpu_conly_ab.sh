#!/bin/bash
# fp8 codes-only MLP outputs: fp8 / block GPU tests, then bench.py --fp8 with APEX_FP8_CODES_ONLY=0 / 1
# interleaved on the same box
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-conly}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py tests/test_post_ln_mem_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
tail -2 $O/pytest.log
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in 0 1; do
    APEX_FP8_CODES_ONLY=$v timeout -k 10 400 python bench.py --steps 10 --warmup 3 --fp8 > $O/b${v}_$r.out 2> $O/b${v}_$r.err
    python -c "import json;d=json.loads(open('$O/b${v}_$r.out').read().strip().splitlines()[-1]);print('codes_only=$v', d['value'], d['fp8']['ms_per_step'], d['fp8']['speedup_vs_bf16'], d['fp8'].get('peak_mem_gb'))"
  done
done
echo done
