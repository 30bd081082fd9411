#!/bin/bash
# Counter-measured HBM traffic of the BERT-shape attention kernels (b768 s128 h16 d64, p = 0.1):
# FETCH_SIZE and WRITE_SIZE in rocprofv3 passes of their own (FETCH_SIZE takes 3 of the 4 TCC
# counter slots, WRITE_SIZE 2), --kernel-trace only; summary by tools/pmc_bw_summary.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-attn_bytes}
mkdir -p $O
timeout -k 10 200 python tools/attn_bench.py --only bert768 > $O/timing.jsonl 2> $O/timing.err || exit 2
i=0
for P in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE"; do
  i=$((i+1))
  for pas in fwd bwd; do
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $O/p${i}_$pas -o p --output-format csv -- python tools/attn_one.py bert768 $pas 0.1 4 > $O/p${i}_$pas.log 2>&1 || { echo "pass $i $pas failed"; tail -5 $O/p${i}_$pas.log; exit 3; }
  done
done
python tools/pmc_bw_summary.py $O > $O/summary.json && cat $O/summary.json
