#!/bin/bash
# rocprofv3 counter passes over tools/bw_kernels.py (each pass its own run, --kernel-trace only;
# FETCH_SIZE takes 3 of the 4 TCC slots, WRITE_SIZE 2, so they cannot share a pass)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-pmc_bw}
OPS=${OPS:-ln,bdaln,lamb,xent,syncbn,syncbn_nhwc,scale}
mkdir -p $O
timeout -k 10 300 python tools/bw_kernels.py --ops $OPS --iters 10 > $O/timing.jsonl 2> $O/timing.err || exit $?
i=0
for P in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $P -d $O/p$i -o p --output-format csv -- python tools/bw_kernels.py --ops $OPS --iters 2 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 3; }
done
python tools/pmc_bw_summary.py $O > $O/summary.json && cat $O/summary.json
