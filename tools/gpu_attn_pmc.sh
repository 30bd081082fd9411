#!/bin/bash
# RCCL same-GPU feasibility + rocprofv3 counter passes on the attention fwd/bwd kernels
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-apmc}
mkdir -p $O
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  tools/rccl_dup_test.py > $O/rccl_dup.log 2>&1; echo "rccl dup rc=$?" >> $O/rccl_dup.log
tail -3 $O/rccl_dup.log
i=0
for P in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  for CASE in "bert bwd 0.1" "gpt2 bwd 0.0" "gpt2 fwd 0.1"; do set -- $CASE
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $O/$1_$2_p$i -o p --output-format csv -- python tools/attn_one.py $1 $2 $3 5 > $O/$1_$2_p$i.log 2>&1 || { echo "pass $i $CASE failed"; tail -5 $O/$1_$2_p$i.log; exit 3; }
  done
done
echo "all done"
