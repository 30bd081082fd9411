#!/bin/bash
# ResNet-50 step kernel table (rocprofv3 kernel trace, last step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${OUT:-profrn}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/r -o run --output-format csv -- python benchmarks/resnet50.py --steps 2 --warmup 1 $RN_ARGS > $O/r.log 2>&1 || { tail -20 $O/r.log; exit 9; }
f=$(find $O/r -name "*kernel_trace.csv" | head -1); python tools/profstep.py $f 1 40 sgd_kernel > $O/rn_step.txt; rm -f $f
cut -c1-170 $O/rn_step.txt
