#!/bin/bash
# Own persistent GEMM vs hipBLASLt at the BERT plain / bias shapes and 8192^3: rocprofv3 counter passes
# (one pass per counter group: the SQ / TCC slot limits) over tools/gemm_energy_vs_lib.py run, then
# the power / energy loops; summary -> $O/pmc_summary.json (median per kernel and counter)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-gpmc}
export O
mkdir -p $O
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SMEM" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
         "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $O/p$i -o p --output-format csv -- python tools/gemm_energy_vs_lib.py run 3 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 3; }
done
python tools/pmc_gemm_summary.py $O > $O/pmc_summary.json && cat $O/pmc_summary.json
timeout -k 10 300 python tools/gemm_energy_vs_lib.py power 2 > $O/power.jsonl 2> $O/power.err || { tail -5 $O/power.err; exit 4; }
cat $O/power.jsonl
