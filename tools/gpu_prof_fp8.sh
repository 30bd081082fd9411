#!/bin/bash
# rocprofv3 kernel trace of bench.py --fp8 (the fp8 pass runs after the bf16 one: tools/profstep.py
# on the trace's last steps reads the fp8 step)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-proff8}
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/bert -o prof --output-format csv -- python bench.py --steps 5 --warmup 2 --fp8 > $O/bert.json 2> $O/bert.err || exit 3
tail -c 300 $O/bert.json
echo "all done"
