#!/bin/bash
# Round-3 validation: GPU test suite, smoke, headline bench, Megatron bench (fp32 main_grad vs
# the bf16 .grad accumulation A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3chk}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
tail -3 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 4; }
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py --fp16 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 5; }
cat $O/bench.json | cut -c1-400
timeout -k 10 400 python benchmarks/megatron_gpt.py > $O/meg.json 2> $O/meg.err || { tail -20 $O/meg.err; exit 6; }
timeout -k 10 400 python benchmarks/megatron_gpt.py --bf16-grad-accum > $O/meg_bf16.json 2> $O/meg_bf16.err || { tail -20 $O/meg_bf16.err; exit 7; }
cut -c1-300 $O/meg.json $O/meg_bf16.json
echo "all done"
