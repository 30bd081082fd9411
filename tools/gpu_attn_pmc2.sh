#!/bin/bash
# rocprofv3 counter passes on the flash-attention fwd / bwd kernels at the three model shapes
# (each pass its own run, --kernel-trace only), summarised by tools/pmc_attn_summary.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-apmc2}
mkdir -p $O
i=0
for P in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_COUNT"; do
  i=$((i+1))
  for CASE in "bert fwd 0.1" "bert bwd 0.1" "gpt2 fwd 0.1" "gpt2 bwd 0.1" "megatron fwd 0.1" "megatron bwd 0.1"; do set -- $CASE
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $O/$1_$2_p$i -o p --output-format csv -- python tools/attn_one.py $1 $2 $3 4 > $O/$1_$2_p$i.log 2>&1 || { echo "pass $i $CASE failed"; tail -5 $O/$1_$2_p$i.log; exit 3; }
  done
done
python tools/pmc_attn_summary.py $O > $O/summary.json && cat $O/summary.json
