#!/bin/bash
# full GPU test suite, smoke(), then the headline bench (and optional extra benches in $BENCHES)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-full}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 4; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 5; }
cat $O/bench.json
i=0
for B in $BENCHES; do i=$((i+1))
  timeout -k 10 400 python benchmarks/$B.py > $O/b_$B.json 2> $O/b_$B.err || { tail -20 $O/b_$B.err; exit 6; }
  cat $O/b_$B.json
done
echo "all done"
