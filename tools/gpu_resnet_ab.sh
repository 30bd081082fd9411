#!/bin/bash
# SyncBN tests, then ResNet-50 interleaved: A fused BN+add+ReLU (default) / B --no-fuse-bn /
# C fused + the step replayed as a HIP graph (--graph); VARIANTS="A C" picks a subset
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-rnab}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_syncbn.py tests/test_models.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in ${VARIANTS:-A B C}; do
    X=""; [ $v = B ] && X="--no-fuse-bn"; [ $v = C ] && X="--graph"
    timeout -k 10 400 python benchmarks/resnet50.py $X > $O/rn_${v}$rep.json 2> $O/rn_${v}$rep.err || { tail -5 $O/rn_${v}$rep.err; exit 4; }
    echo "$v rn50 $(python -c "import json;d=json.load(open('$O/rn_${v}$rep.json'));print(d['value'], d['ms_per_step'], d.get('hip_graph'), d.get('final_loss'))")"
  done
done
echo "all done"
