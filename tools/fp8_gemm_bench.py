"""FP8 vs BF16 GEMM throughput on the hand-written MFMA kernel (csrc/gemm.hip), BERT-large
layer shapes, plus the cost of the per-tensor quantisation that feeds the fp8 path.

    python tools/fp8_gemm_bench.py [--m 16384] [--iters 50]

One JSON line per shape: bf16 / fp8 TFLOP/s (GEMM only) and the quantise time of the activation.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    import apex._ext as e

    C = e.require()
    M = args.m
    one = torch.ones(1, device="cuda")
    for name, N, K in [("qkv", 3072, 1024), ("attn_out", 1024, 1024), ("fc1", 4096, 1024), ("fc2", 1024, 4096),
                       ("dgrad_fc1", 1024, 4096), ("square8k", 8192, 8192)]:
        m = M if name != "square8k" else 8192
        a = torch.randn(m, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
        a8, w8 = C.fp8_quantize(a, 0, one), C.fp8_quantize(w, 0, one * 100)
        t_bf = _time(lambda: C.gemm(a, w, C.EPI_NONE), args.iters)
        t_f8 = _time(lambda: C.gemm_f8(a8, w8, one, one, 0, C.EPI_NONE), args.iters)
        amax = torch.zeros(1, device="cuda")
        t_q = _time(lambda: C.fp8_quantize(a, 0, one, amax), args.iters)
        fl = 2.0 * m * N * K
        print(json.dumps({"shape": name, "M": m, "N": N, "K": K, "bf16_ms": round(t_bf, 4), "fp8_ms": round(t_f8, 4),
                          "bf16_tflops": round(fl / t_bf / 1e9, 1), "fp8_tflops": round(fl / t_f8 / 1e9, 1),
                          "quant_act_ms": round(t_q, 4),
                          "quant_act_GBps": round(a.numel() * 3 / t_q / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
