#!/bin/bash
# Attention GPU tests on the in-tree build, then tools/attn_bench.py interleaved A B A B:
# A = in-tree apex/_C*.so, B = $SO_B (same box). Usage: OUT=name SO_B=abso/_C_base.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-attnab}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 5 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_attention_ext_gpu.py tests/test_multihead_attn.py -m gpu > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 5 200 python tools/attn_bench.py ${ONLY:+--only $ONLY} > $O/A$r.jsonl 2> $O/A$r.err || { tail -5 $O/A$r.err; exit 5; }
  APEX_EXT_SO=$SO_B timeout -k 5 200 python tools/attn_bench.py ${ONLY:+--only $ONLY} > $O/B$r.jsonl 2> $O/B$r.err || { tail -5 $O/B$r.err; exit 6; }
done
python - "$O" <<'PY'
import json, sys, collections
o = sys.argv[1]
rows = collections.defaultdict(dict)
for v in ("A1", "B1", "A2", "B2"):
    for l in open(f"{o}/{v}.jsonl"):
        d = json.loads(l)
        rows[(d["shape"], d["p"], d["pass"])][v] = d["us"]
for k, d in rows.items():
    print(k, " ".join(f"{v}={d.get(v)}" for v in ("A1", "B1", "A2", "B2")))
PY
echo "all done"
