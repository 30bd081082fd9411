"""fp8 weight gradients (csrc/gemm.hip gemm_tt_f8: ds_read_b64_tr_b8 transposed-read main loop over
the uint8 codes, fp32 slabs + splitk_reduce) against the bf16 production path
(apex.ops.fused._wgrad), at BERT-Large's headline batch (M = 98304 tokens), same process,
interleaved rounds.

    python tools/wgrad_f8_bench.py > profiles/r5_wgrad_f8.jsonl

One JSON line per (shape, path): us per call (median of 5 rounds of 10), PF/s, and the error of
the fp8 result against an fp32 product of the dequantised codes (the kernel's own arithmetic) and
against the bf16 product of the unquantised tensors (what quantisation costs).
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _codes(x, dt):
    s = (torch.finfo(dt).max / x.abs().max().float()).reshape(1)
    return (x.float() * s).to(dt).view(torch.uint8), (1.0 / s).float()


def main():
    import argparse

    from apex import _ext
    from apex.ops import fused

    C = _ext.require()
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=98304)
    ap.add_argument("--shapes", default="qkv:3072x1024,attn_out:1024x1024,ffn1:4096x1024,ffn2:1024x4096")
    ap.add_argument("--splits", default="2,4,8,16")
    args = ap.parse_args()
    M = args.M
    torch.manual_seed(0)
    for item in args.shapes.split(","):
        name, nk = item.split(":")
        n, k = (int(v) for v in nk.split("x"))
        dy = torch.randn(M, n, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(M, k, device="cuda", dtype=torch.bfloat16)
        d8, sd = _codes(dy, torch.float8_e5m2)
        x8, sx = _codes(x, torch.float8_e4m3fn)
        out = torch.empty(n, k, device="cuda", dtype=torch.bfloat16)
        ref8 = (d8.view(torch.float8_e5m2).float() * sd).t() @ (x8.view(torch.float8_e4m3fn).float() * sx)
        ref = dy.float().t() @ x.float()
        paths = {"bf16": lambda: fused._wgrad(dy, x, out=out)}
        for s in (int(v) for v in args.splits.split(",")):
            if C.gemm_tt_f8_supported(d8, x8, s):
                paths[f"f8_s{s}"] = (lambda s=s: C.gemm_tt_f8(d8, x8, sd, sx, 1, 0, s, torch.bfloat16, out=out))
        err = {}
        for p, f in paths.items():
            f()
            o = out.float()
            err[p] = (float((o - ref8).abs().max() / ref8.abs().max()), float((o - ref).norm() / ref.norm()))
        res = {p: [] for p in paths}
        for _ in range(5):
            for p, f in paths.items():
                f()
                torch.cuda.synchronize()
                e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                e[0].record()
                for _ in range(10):
                    f()
                e[1].record()
                torch.cuda.synchronize()
                res[p].append(e[0].elapsed_time(e[1]) * 100.0)
        for p in paths:
            us = statistics.median(res[p])
            print(json.dumps({"shape": name, "M": M, "N": n, "K": k, "path": p, "us": round(us, 1),
                              "pflops": round(2.0 * M * n * k / us / 1e9, 3),
                              "rel_max_err_vs_dequant_fp32": err[p][0], "rel_fro_err_vs_bf16_inputs": err[p][1]}),
                  flush=True)
        del dy, x, d8, x8, out, ref8, ref


if __name__ == "__main__":
    main()
