#!/bin/bash
# rocprofv3 counter passes (each its own run, --kernel-trace only) on one GEMM shape
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-pmc}
mkdir -p $O
SHAPE=${SHAPE:-"32768 1024 4096 0 0 10"}
i=0
for P in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $O/p$i -o p --output-format csv -- python tools/gemm_one.py $SHAPE > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 3; }
  [ -n "$SHAPE2" ] && { timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $O/q$i -o p --output-format csv -- python tools/gemm_one.py $SHAPE2 > $O/q$i.log 2>&1 || { echo "pass q$i failed"; exit 3; }; }
done
echo "all done"
