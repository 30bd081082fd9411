#!/bin/bash
# round 4: BERT-Large b768 step kernel table, balanced GEMM loop tree
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/g31prof -o prof --output-format csv -- python bench.py --steps 4 --warmup 3 --no-fp32 > $O/g31_prof_bench.json 2> $O/g31_prof.err || exit 1
f=$(find $O/g31prof -name "*kernel_trace.csv" | head -1)
python tools/profstep.py "$f" 3 60 > $O/g31_step_kernels.txt
rm -rf $O/g31prof
head -5 $O/g31_step_kernels.txt
