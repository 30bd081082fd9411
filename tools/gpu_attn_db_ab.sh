set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/attdb
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 5 300 python -m pytest -q -x --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_attention_ext_gpu.py tests/test_multihead_attn.py -m gpu > $O/t_db.log 2>&1 || { tail -20 $O/t_db.log; exit 3; }
tail -1 $O/t_db.log
APEX_EXT_SO=abso/_C_w3.so timeout -k 5 300 python -m pytest -q -x --timeout 120 --timeout-method thread tests/test_attention_gpu.py -m gpu > $O/t_w3.log 2>&1 || { tail -20 $O/t_w3.log; exit 4; }
tail -1 $O/t_w3.log
for r in 1 2; do
  APEX_ATTN_FWD_DB=0 timeout -k 5 200 python tools/attn_bench.py > $O/old$r.jsonl || exit 5
  timeout -k 5 200 python tools/attn_bench.py > $O/db$r.jsonl || exit 6
  APEX_EXT_SO=abso/_C_w3.so timeout -k 5 200 python tools/attn_bench.py > $O/w3$r.jsonl || exit 7
done
grep -h '"fwd"' $O/old1.jsonl $O/db1.jsonl $O/w31.jsonl $O/old2.jsonl $O/db2.jsonl $O/w32.jsonl
