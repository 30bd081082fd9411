#!/bin/bash
# round 4: first-round GEMM stagger re-test with the balanced loop (bench A/B, same box)
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
: > $O/g28_stagger.jsonl
for st in "" "8:2" "8:4" "4:2,10:2" "" ; do
  APEX_GEMM_STAGGER="$st" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-fp32 > $O/g28_b.json 2> $O/g28_b.err || { tail $O/g28_b.err; exit 1; }
  python -c "import json,sys;d=json.load(open('$O/g28_b.json'));print(json.dumps({'stagger':sys.argv[1],'value':d['value'],'ms':d['ms_per_step'],'sclk':d['gpu']['timed']['sclk_mhz']['mean']}))" "$st" >> $O/g28_stagger.jsonl
done
cat $O/g28_stagger.jsonl
