#!/bin/bash
# where the fp32 main_grad mode's CUDAFunctor_add<float> launches come from (grid-size histogram)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${OUT:-megadds}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/t -o run --output-format csv -- python benchmarks/megatron_gpt.py --steps 1 --warmup 1 --layers 4 > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 8; }
f=$(find $O/t -name "*kernel_trace.csv" | head -1)
python tools/trace_sizes.py $f CUDAFunctor_add FillFunctor > $O/sizes.txt
rm -f $f
cat $O/sizes.txt
