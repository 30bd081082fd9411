#!/bin/bash
# rocprofv3 kernel stats of the headline BERT-Large step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-profb}
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/bert -o prof --output-format csv -- python bench.py --steps 5 --warmup 2 > $O/bert.json 2> $O/bert.err || exit 3
cat $O/bert.json
echo "all done"
