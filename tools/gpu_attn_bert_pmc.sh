#!/bin/bash
# BERT-shape attention (SHAPE: bert = b256 s128 h16 d64, bert768 = b768; p 0.1): timing + where the
# waves spend their cycles
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-bpmc}
SHAPE=${SHAPE:-bert}
export O
mkdir -p $O
timeout -k 10 200 python tools/attn_bench.py --only $SHAPE > $O/bench.jsonl 2> $O/bench.err || { tail -5 $O/bench.err; exit 2; }
cat $O/bench.jsonl
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
         "FETCH_SIZE GRBM_COUNT"; do
  i=$((i+1))
  for pas in fwd bwd; do
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $O/${pas}_p$i -o p --output-format csv -- python tools/attn_one.py $SHAPE $pas 0.1 4 > $O/${pas}_p$i.log 2>&1 || { echo "pass $i $pas failed"; tail -5 $O/${pas}_p$i.log; exit 3; }
  done
done
python - <<'PY'
import csv, glob, json, collections, os
out = {}
O = os.environ["O"]
for f in glob.glob(O + "/*_p*/**/*counter_collection.csv", recursive=True):
    pas = os.path.relpath(f, O).split("/")[0].split("_")[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "attn_" not in r["Kernel_Name"] or "delta" in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        v.sort()
        out.setdefault(pas, {})[k] = v[len(v) // 2]
json.dump(out, open(O + "/pmc_summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
