#!/bin/bash
# Megatron GPT step tables (rocprofv3 kernel trace, last step): fp32 main_grad vs bf16 .grad
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${OUT:-megprof2}
mkdir -p $O
for mode in p32 p16; do
  extra=""; [ $mode = p16 ] && extra="--bf16-grad-accum"
  timeout -k 10 400 rocprofv3 --kernel-trace -d $O/$mode -o run --output-format csv -- python benchmarks/megatron_gpt.py --steps 2 --warmup 1 $extra > $O/$mode.log 2>&1 || { tail -20 $O/$mode.log; exit 8; }
  f=$(find $O/$mode -name "*kernel_trace.csv" | head -1)
  python tools/profstep.py $f 1 28 adam_kernel > $O/${mode}_step.txt
  rm -f $f
  cut -c1-190 $O/${mode}_step.txt
done
echo "all done"
