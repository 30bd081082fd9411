#!/bin/bash
# rocprofv3 kernel traces of the GPT-2 1.5B and Megatron GPT benches (per-step breakdown by tools/profstep.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-profgm}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/gpt2 -o prof --output-format csv -- python benchmarks/gpt2.py --steps 3 --warmup 1 > $O/gpt2.json 2> $O/gpt2.err || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/meg -o prof --output-format csv -- python benchmarks/megatron_gpt.py --steps 2 --warmup 1 --global-batch 8 > $O/meg.json 2> $O/meg.err || exit 4
for m in gpt2 meg; do f=$(find $O/$m -name "*kernel_trace.csv" | head -1); python tools/profstep.py $f 2 25 adam > $O/${m}_steps.txt; head -30 $O/${m}_steps.txt; done
echo "all done"
