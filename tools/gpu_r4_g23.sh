#!/bin/bash
# round 4: weight-gradient (TR) GEMM lab at the BERT-Large shapes + an LDS counter pass
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
: > $O/g23_trlab.jsonl
for sh in "3072 1024" "1024 1024" "4096 1024" "1024 4096"; do
  for s in 4 8 16; do
    timeout -k 10 60 labbin/trlab $sh 98304 $s 3 5 >> $O/g23_trlab.jsonl || { echo "trlab $sh $s failed"; exit 2; }
  done
done
P="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $O/g23pmc -o p --output-format csv -- labbin/trlab 3072 1024 98304 16 1 1 > $O/g23_pmc.log 2>&1 || { echo "pmc failed"; exit 3; }
f=$(find $O/g23pmc -name "*counter_collection.csv" | head -1)
python tools/pmc_sum.py "$f" > $O/g23_pmc.txt 2>&1 || cp "$f" $O/g23_pmc_raw.csv
rm -rf $O/g23pmc
cat $O/g23_trlab.jsonl
