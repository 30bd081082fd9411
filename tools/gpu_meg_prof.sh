#!/bin/bash
# Megatron GPT step: fp32 main_grad vs bf16 .grad accumulation, timed and kernel-traced
# (rocprofv3 --kernel-trace --stats), so the two step tables can be diffed.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-megprof}
mkdir -p $O
export PYTHONUNBUFFERED=1
[ -n "$NOTIME" ] || timeout -k 10 400 python benchmarks/megatron_gpt.py > $O/meg.json 2> $O/meg.err || { tail -20 $O/meg.err; exit 6; }
[ -n "$NOTIME" ] || timeout -k 10 400 python benchmarks/megatron_gpt.py --bf16-grad-accum > $O/meg_bf16.json 2> $O/meg_bf16.err || { tail -20 $O/meg_bf16.err; exit 7; }
[ -n "$NOTIME" ] || cut -c1-300 $O/meg.json $O/meg_bf16.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/p32 -o run --output-format csv -- python benchmarks/megatron_gpt.py --steps 2 --warmup 1 > $O/p32.log 2>&1 || { tail -20 $O/p32.log; exit 8; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/p16 -o run --output-format csv -- python benchmarks/megatron_gpt.py --steps 2 --warmup 1 --bf16-grad-accum > $O/p16.log 2>&1 || { tail -20 $O/p16.log; exit 9; }
for f in $(find $O -name "*kernel_trace.csv"); do python tools/trace_sizes.py $f CUDAFunctor_add FillFunctor copyBuffer > ${f%.csv}_sizes.txt; done
find $O -name "*kernel_trace.csv" -delete
cat $(find $O -name "*_sizes.txt")
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; head -25 "$f" | cut -c1-200; done
echo "all done"
