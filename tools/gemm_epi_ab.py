"""Fused-epilogue MFMA GEMMs of a BERT-Large layer at the headline batch (M = 98304 tokens by
default, PB_M to change): us per call, best of 3 interleaved rounds, one JSON line per case.
Run it under two builds of the extension (APEX_EXT_SO) for a same-box A/B of a kernel change.

  python tools/gemm_epi_ab.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.gemm_mfma_bench import bench  # noqa: E402


def r(*s):
    return torch.empty(*s, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)


def main():
    import apex._ext as e

    C = e.require()
    M = int(os.environ.get("PB_M", 98304))
    H, F = 1024, 4096
    x, g = r(M, H), r(M, F)
    wqkv, w1, w2 = r(3 * H, H) * 0.03, r(F, H) * 0.03, r(H, F) * 0.03
    bqkv, b1 = r(3 * H), r(F)
    dt, dqkv, dh, gd, dres = r(M, H), r(M, 3 * H), r(M, F), r(M, F), r(M, H)
    wqkvT, w1T, w2T = (C.transpose(w) for w in (wqkv, w1, w2))
    cases = {
        "ffn1_fwd_gelu_d": lambda: C.gemm(x, w1, 8, b1),
        "ffn2_dgrad_mul": lambda: C.gemm(dt, w2T, 10, None, gd, torch.bfloat16),
        "qkv_dgrad_resid": lambda: C.gemm(dqkv, wqkvT, 4, None, dres),
        "ffn1_dgrad_resid": lambda: C.gemm(dh, w1T, 4, None, dres),
        "qkv_fwd_bias": lambda: C.gemm(x, wqkv, 1, bqkv),
        "ffn2_fwd_plain": lambda: C.gemm(g, w2, 0),
    }
    flops = {"ffn1_fwd_gelu_d": 2 * M * F * H, "ffn2_dgrad_mul": 2 * M * F * H, "qkv_dgrad_resid": 2 * M * H * 3 * H,
             "ffn1_dgrad_resid": 2 * M * H * F, "qkv_fwd_bias": 2 * M * 3 * H * H, "ffn2_fwd_plain": 2 * M * H * F}
    best = {k: 1e30 for k in cases}
    for _ in range(3):
        for k, fn in cases.items():
            best[k] = min(best[k], bench(fn))
    for k, v in best.items():
        print(json.dumps({"case": k, "M": M, "us": round(v, 1), "tflops": round(flops[k] / v / 1e6, 1),
                          "so": os.path.basename(os.environ.get("APEX_EXT_SO", "in-tree"))}), flush=True)


if __name__ == "__main__":
    main()
