"""BERT-Large weight-gradient GEMMs at the headline batch (M = 98304 tokens): the production path
(apex.ops.fused._wgrad: fp32-output batched split-K GEMM + one HIP reduction) vs ONE TunableOp-tuned
library GEMM dW = dY^T X in bf16 (hipBLASLt's own split-K / stream-K solutions included in the
search). Tuning runs here, into ``--out`` (a TunableOp results file), never inside a timed run.

  python tools/wgrad_tune_bench.py --out gpurun_out/wgrad_tune/tunableop_results%d.csv

One JSON line per (shape, path): us per call.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters=10, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(iters):
        fn()
    e[1].record()
    torch.cuda.synchronize()
    return e[0].elapsed_time(e[1]) / iters * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--M", type=int, default=98304)
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    from apex.ops.fused import _wgrad

    M = a.M
    shapes = {"qkv": (3072, 1024), "attn_out": (1024, 1024), "ffn1": (4096, 1024), "ffn2": (1024, 4096)}
    data = {k: (torch.randn(M, n, device="cuda", dtype=torch.bfloat16), torch.randn(M, kk, device="cuda",
                                                                                   dtype=torch.bfloat16))
            for k, (n, kk) in shapes.items()}
    for name, (dy, x) in data.items():
        print(json.dumps({"shape": name, "M": M, "N": dy.shape[1], "K": x.shape[1], "path": "production_splitk",
                          "us": round(timed(lambda: _wgrad(dy, x)), 1)}), flush=True)
    import torch.cuda.tunable as tun

    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(a.out)
    tun.set_max_tuning_duration(30)
    tun.set_max_tuning_iterations(20)
    for name, (dy, x) in data.items():
        torch.mm(dy.t(), x)  # tunes this shape
        torch.cuda.synchronize()
    tun.tuning_enable(False)
    for name, (dy, x) in data.items():
        us = timed(lambda: torch.mm(dy.t(), x))
        err = float((torch.mm(dy.t(), x).float() - _wgrad(dy, x).float()).abs().max())
        print(json.dumps({"shape": name, "M": M, "N": dy.shape[1], "K": x.shape[1], "path": "tuned_single_gemm",
                          "us": round(us, 1), "max_abs_diff_vs_production": err}), flush=True)
    # (TunableOp writes the results file at exit)


if __name__ == "__main__":
    main()
