#!/bin/bash
# round 4: trainable attention bias through the flash kernels (dS written / atomically added into the
# bias gradient), attention test files
set -o pipefail
O=gpurun_out/r4; mkdir -p $O
T="timeout -k 10"
PT="python -u -m pytest -q -x --timeout 120 --timeout-method thread"
$T 500 $PT tests/test_attention_bias_grad_gpu.py tests/test_attention_fp32_gpu.py tests/test_attention_gpu.py tests/test_attention_ext_gpu.py tests/test_attention_f32_kernel_gpu.py tests/test_context_parallel_gpu.py > $O/g12_tests.log 2>&1 || exit 1
echo done
