#!/bin/bash
# round 4: forward dropout applied to the packed P operand (byte masks + v_perm): attention tests,
# BERT-shape microbench, VALU/MFMA counters of the forward
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
T="timeout -k 10"
PT="python -u -m pytest -q -x --timeout 120 --timeout-method thread"
$T 400 $PT tests/test_attention_gpu.py tests/test_attention_ext_gpu.py tests/test_attention_f32_kernel_gpu.py > $O/g8_tests.log 2>&1 || exit 1
$T 120 python tools/attn_bench.py --only bert768 > $O/g8_attn.jsonl 2>/dev/null || exit 1
$T 120 python tools/attn_bench.py --only bert768 >> $O/g8_attn.jsonl 2>/dev/null || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P1 -d $O/g8pmc/fwd_p1 -o p --output-format csv -- python tools/attn_one.py bert768 fwd 0.1 4 > $O/g8pmc_fwd_p1.log 2>&1 || { echo "pmc failed"; exit 3; }
python - <<'PY' > $O/g8_attn_pmc.json
import csv, glob, json, collections
out = {}
for f in glob.glob("gpurun_out/r4/g8pmc/*_p*/**/*counter_collection.csv", recursive=True):
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
rm -rf $O/g8pmc
bash tools/gpu_r4_g9.sh || exit 1
