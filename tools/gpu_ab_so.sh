#!/bin/bash
# Same-box A/B of two builds of the extension: the in-tree apex/_C*.so (A) vs $SO_B (B),
# interleaved A B A B on the headline bench and the benches in $BENCHES.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-absos}
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for v in A B; do
    if [ $v = B ]; then X="${B_ENV:-APEX_EXT_SO=$SO_B}"; else X="APEX_AB=A"; fi
    env $X timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bert_${v}$rep.json 2> $O/bert_${v}$rep.err || { tail -5 $O/bert_${v}$rep.err; exit 3; }
    echo "$v bert $(python -c "import json;d=json.load(open('$O/bert_${v}$rep.json'));print(d['value'], d['ms_per_step'])")"
    for B in $BENCHES; do
      env $X timeout -k 10 400 python benchmarks/$B.py > $O/${B}_${v}$rep.json 2> $O/${B}_${v}$rep.err || { tail -5 $O/${B}_${v}$rep.err; exit 4; }
      echo "$v $B $(python -c "import json;d=json.load(open('$O/${B}_${v}$rep.json'));print(d['value'], d['ms_per_step'])")"
    done
  done
done
echo "all done"
