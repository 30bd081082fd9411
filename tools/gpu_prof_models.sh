#!/bin/bash
# rocprofv3 kernel stats of the GPT-2 1.5B and ResNet-50 benches
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-profm}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/gpt2 -o prof --output-format csv -- python benchmarks/gpt2.py --steps 3 --warmup 1 > $O/gpt2.json 2> $O/gpt2.err || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/rn50 -o prof --output-format csv -- python benchmarks/resnet50.py --steps 4 --warmup 2 > $O/rn50.json 2> $O/rn50.err || exit 4
echo "all done"
