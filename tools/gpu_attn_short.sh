#!/bin/bash
# attention tests, the BERT-shape attention microbench for the in-tree build (A) and $SO_B (B),
# then the same-box A/B of the headline step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-attnshort}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_multihead_attn.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -2 $O/pytest.log
timeout -k 10 200 python tools/attn_bench.py --only bert > $O/attn_A.jsonl 2> $O/attn_A.err || { tail -5 $O/attn_A.err; exit 4; }
APEX_EXT_SO=$SO_B timeout -k 10 200 python tools/attn_bench.py --only bert > $O/attn_B.jsonl 2> $O/attn_B.err || { tail -5 $O/attn_B.err; exit 5; }
echo A; cat $O/attn_A.jsonl; echo B; cat $O/attn_B.jsonl
OUT=${OUT:-attnshort} bash tools/gpu_ab_so.sh
