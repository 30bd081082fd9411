#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
O=gpurun_out/attn2
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/attn_bench.py > $O/attn.jsonl 2> $O/attn.err; rc=$?; cat $O/attn.jsonl
[ $rc -eq 0 ] || exit 3
timeout -k 10 600 python -m pytest tests/test_fused_ops_gpu.py -m gpu -q -rf -k "sublayer or wgrad" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json
[ $rc -eq 0 ] || exit 5
APEX_BERT_SUBLAYER_FUSION=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_nofuse.json 2> $O/bench_nofuse.err; rc=$?; cat $O/bench_nofuse.json
[ $rc -eq 0 ] || exit 6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVES -d $O/pmc -o pmc --output-format csv -- python tools/attn_bench.py --only gpt2 > $O/pmc.out 2>&1 || exit 7
echo "all done"
