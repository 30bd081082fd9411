"""Weight-gradient GEMM dW[N,K] = dY[M,N]^T X[M,K] at the BERT-Large b768 token count (M = 98304):
library batched GEMM over S token slices + the HIP slab reduction, for every S that divides M,
and the hand-written transposed-read MFMA kernel (gemm_tt) at its splits. us per call (best of 3
interleaved rounds), one JSON line per (shape, variant). Picks the split table of _wgrad_splits.

  python tools/wgrad_split_sweep.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.gemm_mfma_bench import bench  # noqa: E402


def main():
    from apex.utils.gemm_tuning import enable_tuned_gemms

    enable_tuned_gemms()
    import apex._ext as e

    C = e.require()
    M = int(os.environ.get("PB_M", 98304))
    shapes = {"qkv": (3072, 1024), "o": (1024, 1024), "ffn1": (4096, 1024), "ffn2": (1024, 4096)}
    for name, (N, K) in shapes.items():
        dy = torch.empty(M, N, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        cases = {}
        for s in (1, 2, 3, 4, 6, 8, 12, 16, 24, 32):
            if M % s:
                continue
            if s == 1:
                cases["lib_s1"] = lambda: torch.mm(dy.t(), x, out=out)
            else:
                def f(s=s):
                    slabs = torch.bmm(dy.view(s, M // s, N).transpose(1, 2), x.view(s, M // s, K),
                                      out_dtype=torch.float32)
                    C.splitk_reduce(slabs, dy.dtype, out)
                cases[f"lib_s{s}"] = f
        for s in (2, 4, 8, 16):
            if C.gemm_tt_supported(dy, x, s):
                cases[f"tt_s{s}"] = lambda s=s: C.gemm_tt(dy, x, s, dy.dtype)
        best = {k: 1e30 for k in cases}
        for _ in range(3):
            for k, fn in cases.items():
                best[k] = min(best[k], bench(fn, iters=10, warm=3))
        fl = 2.0 * M * N * K
        for k, v in sorted(best.items(), key=lambda kv: kv[1]):
            print(json.dumps({"shape": name, "N": N, "K": K, "M": M, "variant": k, "us": round(v, 1),
                              "tflops": round(fl / v / 1e6, 1)}), flush=True)
        del dy, x, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
