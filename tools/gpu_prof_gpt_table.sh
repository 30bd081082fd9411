#!/bin/bash
# rocprofv3 kernel traces of the GPT-2 1.5B step with the weight gradients on the library
# (APEX_WGRAD_TT_TABLE=none) and on the transposed-read kernel (GPT table), then the BERT A/B rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-profgt}
mkdir -p $O
GPT=${GPT_TABLE:-"1600x1600:16384:4,6400x1600:16384:4,1600x6400:16384:4"}
for t in none tab; do
  if [ $t = none ]; then export APEX_WGRAD_TT_TABLE=none; else export APEX_WGRAD_TT_TABLE="$GPT"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/gpt_$t -o prof --output-format csv -- python benchmarks/gpt2.py --steps 5 --warmup 2 > $O/gpt_$t.json 2> $O/gpt_$t.err || exit 3
done
unset APEX_WGRAD_TT_TABLE
for r in 1 2 3; do
  APEX_WGRAD_TT_TABLE="1024x1024:65536:16" timeout -k 10 400 python bench.py > $O/bert_tab_$r.json 2>/dev/null || exit 4
  APEX_WGRAD_TT_TABLE=none timeout -k 10 400 python bench.py > $O/bert_none_$r.json 2>/dev/null || exit 4
done
echo "all done"
