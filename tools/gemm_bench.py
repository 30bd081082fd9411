"""GEMM microbenchmark for the BERT-Large weight-gradient shapes: dW[N,K] = dY[M,N]^T @ X[M,K]
with M = tokens (32768). Compares the library call against split-K batched variants (fp32
partials via bmm(out_dtype=fp32) + reduction). Interleaved rounds in one process.

  python tools/gemm_bench.py [--m 32768]
"""
import argparse
import json

import torch


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
    return ev[0].elapsed_time(ev[1]) / iters * 1000.0  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=32768)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    M = a.m
    shapes = [(1024, 1024), (3072, 1024), (4096, 1024), (1024, 4096)]  # (N, K): dY [M,N], X [M,K]
    res = []
    for N, K in shapes:
        dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        flops = 2.0 * M * N * K
        ref = (dy.float().t() @ x.float())
        variants = {"mm": lambda: dy.t() @ x}
        for s in (2, 4, 8, 16):
            if M % s:
                continue

            def f(s=s):
                p = torch.bmm(dy.view(s, M // s, N).transpose(1, 2), x.view(s, M // s, K), out_dtype=torch.float32)
                return p.sum(0)

            variants[f"splitk{s}"] = f
        for name, fn in variants.items():
            out = fn().float()
            err = float((out - ref).abs().max() / ref.abs().max())
            ts = [bench(fn) for _ in range(a.rounds)]
            t = min(ts)
            res.append({"N": N, "K": K, "variant": name, "us": round(t, 1), "tflops": round(flops / t / 1e6, 1),
                        "rel_err": err})
            print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()
