#!/bin/bash
# GEMM GPU tests with the in-tree build, then a same-box A/B of the fused-epilogue GEMMs:
# in-tree apex/_C*.so (A) vs $SO_B (B), interleaved A B A B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-gemmab}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_fp8_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
for rep in 1 2; do
  timeout -k 10 200 python tools/gemm_epi_ab.py > $O/A$rep.jsonl 2> $O/A$rep.err || { tail -20 $O/A$rep.err; exit 4; }
  APEX_EXT_SO=$SO_B timeout -k 10 200 python tools/gemm_epi_ab.py > $O/B$rep.jsonl 2> $O/B$rep.err || { tail -20 $O/B$rep.err; exit 5; }
done
cat $O/A*.jsonl $O/B*.jsonl
echo "all done"
