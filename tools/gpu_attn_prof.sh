#!/bin/bash
# kernel-trace stats + one counter pass for the attention backward kernels at the long shapes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-aprof}
mkdir -p $O
for CASE in "megatron bwd 0.1" "gpt2 bwd 0.1" "megatron fwd 0.1"; do set -- $CASE
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/st_$1_$2 -o p --output-format csv -- python tools/attn_one.py $1 $2 $3 10 > $O/st_$1_$2.log 2>&1 || { echo "stats $CASE failed"; exit 3; }
done
P="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_ANY"
for CASE in "megatron bwd 0.1" "gpt2 bwd 0.1"; do set -- $CASE
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $O/pmc_$1_$2 -o p --output-format csv -- python tools/attn_one.py $1 $2 $3 4 > $O/pmc_$1_$2.log 2>&1 || { echo "pmc $CASE failed"; exit 4; }
done
P="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for CASE in "megatron bwd 0.1" "gpt2 bwd 0.1"; do set -- $CASE
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $O/pmc2_$1_$2 -o p --output-format csv -- python tools/attn_one.py $1 $2 $3 4 > $O/pmc2_$1_$2.log 2>&1 || { echo "pmc2 $CASE failed"; exit 5; }
done
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-4 "$f" | head -6; done
echo "all done"
