#!/bin/bash
# rocprofv3 kernel trace of the headline step (b768) -> per-step kernel table; optional extra
# command in $EXTRA (run after the profile, output under the same directory).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-prof_step}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/bert -o prof --output-format csv -- python bench.py --steps 4 --warmup 3 --no-fp32 > $O/bert.json 2> $O/bert.err || exit $?
f=$(find $O/bert -name "*kernel_trace.csv" | head -1)
python tools/profstep.py "$f" 3 45 > $O/bert_steps.txt && head -40 $O/bert_steps.txt
rm -f "$f"
if [ -n "$EXTRA" ]; then
  eval "$EXTRA" || exit $?
fi
echo "all done"
