#!/bin/bash
# step kernel tables of the GPT-2 1.5B and ResNet-50 benches (rocprofv3 kernel trace, last step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${OUT:-profothers}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/g -o run --output-format csv -- python benchmarks/gpt2.py --steps 2 --warmup 1 > $O/g.log 2>&1 || { tail -20 $O/g.log; exit 8; }
f=$(find $O/g -name "*kernel_trace.csv" | head -1); python tools/profstep.py $f 1 30 adam_kernel > $O/gpt2_step.txt; rm -f $f
cut -c1-170 $O/gpt2_step.txt
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/r -o run --output-format csv -- python benchmarks/resnet50.py --steps 2 --warmup 1 > $O/r.log 2>&1 || { tail -20 $O/r.log; exit 9; }
f=$(find $O/r -name "*kernel_trace.csv" | head -1); python tools/profstep.py $f 1 30 sgd_kernel > $O/rn_step.txt; rm -f $f
cut -c1-170 $O/rn_step.txt
