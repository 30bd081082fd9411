#!/bin/bash
# round 4: ring-attention one-call-per-step schedule (CP GPU tests + single-GPU emulation) and the
# BERT-shape attention PMC passes at b768 after the stream RNG / backward changes
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_context_parallel_gpu.py > $O/g4_cp_tests.log 2>&1 || exit 1
$T 200 python tools/cp_emul_bench.py > $O/g4_cp_emul.jsonl 2> $O/g4_cp_emul.err || exit 1
$T 200 python tools/cp_emul_bench.py --S 16384 >> $O/g4_cp_emul.jsonl 2>> $O/g4_cp_emul.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  for pas in fwd bwd; do
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d $O/g4pmc/${pas}_p$i -o p --output-format csv -- python tools/attn_one.py bert768 $pas 0.1 4 > $O/g4pmc_${pas}_p$i.log 2>&1 || { echo "pass $i $pas failed"; exit 3; }
  done
done
python - <<'PY' > $O/g4_attn_pmc.json
import csv, glob, json, collections
out = {}
for f in glob.glob("gpurun_out/r4/g4pmc/*_p*/**/*counter_collection.csv", recursive=True):
    pas = f.split("/")[3].split("_")[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "attn_" not in r["Kernel_Name"] or "delta" in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        v.sort()
        out.setdefault(pas, {})[k] = v[len(v) // 2]
print(json.dumps(out, indent=1))
PY
rm -rf $O/g4pmc
echo done
