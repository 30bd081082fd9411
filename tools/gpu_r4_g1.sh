set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_fp32_gpu.py tests/test_chunked_attention.py tests/test_fused_ops_gpu.py tests/test_context_parallel_gpu.py tests/test_main_grad_gpu.py > gpurun_out/r4/g1_tests.log 2>&1 &&
timeout -k 10 420 python bench.py --steps 20 --warmup 5 > gpurun_out/r4/g1_bench.json 2> gpurun_out/r4/g1_bench.err
