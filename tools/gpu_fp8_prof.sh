#!/bin/bash
# BERT-Large b768 fp8 step kernel table (rocprofv3 kernel trace; the fp8 pass runs last, so the
# last 2 steps are fp8 steps). APEX_FP8_PRODUCER passes through.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${OUT:-fp8prof}
mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace -d $O/t -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-fp32 --fp8 --fp8-steps 3 > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 8; }
f=$(find $O/t -name "*kernel_trace.csv" | head -1)
python tools/profstep.py $f 2 45 > $O/step.txt
rm -f $f
cut -c1-200 $O/step.txt
