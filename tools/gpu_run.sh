#!/bin/bash
# Chained GPU steps for one gpurun call. Usage: tools/gpu_run.sh OUTDIR "name|timeout|cmd" ...
# A step that exits 0 or 1 (test failures) lets the chain continue; any other status (fault,
# abort, segfault, time limit) stops the chain: nothing more runs on the GPU in this call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
out="gpurun_out/$1"; shift
mkdir -p "$out"
export PYTHONUNBUFFERED=1
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; to="${rest%%|*}"; cmd="${rest#*|}"
  echo "== $name (timeout $to s): $cmd"
  timeout -k 10 "$to" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -4 "$out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping chain after $name (rc=$rc)"; exit $rc; fi
done
