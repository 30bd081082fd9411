#!/bin/bash
# Same-box A/B of weight-gradient routing tables (APEX_WGRAD_TT_TABLE, apex/ops/fused.py) on the
# model steps: BERT-Large (bench.py) with the attention-out shape on the transposed-read kernel at 16
# slices vs the library, and GPT-2 1.5B (benchmarks/gpt2.py) with its attention-out / FFN shapes at 4
# slices vs the library; each interleaved twice.
set -euo pipefail
OUT=gpurun_out/${1:-wgrad_table}
mkdir -p "$OUT"
BERT=${BERT_TABLE:-"1024x1024:65536:16"}
GPT=${GPT_TABLE:-"1600x1600:16384:4,6400x1600:16384:4,1600x6400:16384:4"}
for r in 1 2; do
  APEX_WGRAD_TT_TABLE=none timeout -k 10 400 python bench.py > "$OUT/bert_none_$r.json" 2> "$OUT/bert_none_$r.err"
  APEX_WGRAD_TT_TABLE="$BERT" timeout -k 10 400 python bench.py > "$OUT/bert_tab_$r.json" 2> "$OUT/bert_tab_$r.err"
done
for r in 1 2; do
  APEX_WGRAD_TT_TABLE=none timeout -k 10 400 python benchmarks/gpt2.py > "$OUT/gpt_none_$r.json" 2> "$OUT/gpt_none_$r.err"
  APEX_WGRAD_TT_TABLE="$GPT" timeout -k 10 400 python benchmarks/gpt2.py > "$OUT/gpt_tab_$r.json" 2> "$OUT/gpt_tab_$r.err"
done
