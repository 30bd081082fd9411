"""MFMA GEMM (csrc/gemm.hip) vs the library GEMM (torch.mm -> hipBLASLt) on the BERT-Large
dense-layer shapes, random bf16 data, interleaved rounds in one process.

Forward:  Y[M,N] = X[M,K] W[N,K]^T          (QKV, attn-out, FFN1, FFN2)
Dgrad:    dX[M,K] = dY[M,N] W[N,K]  ==  dY . (W^T)^T   (the MFMA kernel takes W^T, K-contiguous)

  python tools/gemm_mfma_bench.py [--m 32768] [--rounds 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / iters * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=32768)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import apex._ext as e

    C = e.require()
    M = a.m
    shapes = [("qkv", 3072, 1024), ("attn_out", 1024, 1024), ("ffn1", 4096, 1024), ("ffn2", 1024, 4096),
              ("sq4096", 4096, 4096)]
    for name, N, K in shapes:
        x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        w = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        bias = torch.randn(N, device="cuda", dtype=torch.bfloat16)
        flops = 2.0 * M * N * K
        ref = x.float() @ w.float().t()
        out, _ = C.gemm(x, w, C.EPI_NONE)
        err = float((out.float() - ref).abs().max() / ref.abs().max())
        del ref
        variants = {
            "torch.mm": lambda: torch.mm(x, w.t()),
            "torch.addmm": lambda: torch.addmm(bias, x, w.t()),
            "mfma": lambda: C.gemm(x, w, C.EPI_NONE),
            "mfma_bias": lambda: C.gemm(x, w, C.EPI_BIAS, bias),
            "mfma_bias_gelu": lambda: C.gemm(x, w, C.EPI_BIAS_GELU, bias),
        }
        best = {k: 1e30 for k in variants}
        for _ in range(a.rounds):
            for k, fn in variants.items():
                best[k] = min(best[k], bench(fn))
        for k, t in best.items():
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "variant": k, "us": round(t, 1),
                              "tflops": round(flops / t / 1e6, 1), "rel_err": err if k == "mfma" else None}),
                  flush=True)


if __name__ == "__main__":
    main()
