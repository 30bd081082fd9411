"""BERT-Large weight gradients at the headline batch (M = 98304 tokens), in one process and
interleaved: the library split-K path (batched hipBLASLt GEMM into fp32 slabs + splitk_reduce)
against the transposed-read MFMA kernel (csrc/gemm.hip gemm_tt, same slabs + reduce) at 2-16 slices,
both writing a preallocated gradient slot as DDP's buckets do (apex.ops.fused._wgrad).

    python tools/wgrad_tt_bench.py > profiles/r4_wgrad_tt_vs_lib.jsonl

One JSON line per (shape, path): us per call (median of 5 rounds of 10), max |diff| vs the library.
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import argparse

    from apex.ops import fused

    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=98304)
    ap.add_argument("--shapes", default="qkv:3072x1024,attn_out:1024x1024,ffn1:4096x1024,ffn2:1024x4096",
                    help="name:NxK,... (GPT-2 1.5B at M = 16384: qkv:4800x1600,attn_out:1600x1600,"
                         "ffn1:6400x1600,ffn2:1600x6400)")
    ap.add_argument("--splits", default="2,4,8,16")
    ap.add_argument("--untuned", action="store_true",
                    help="library GEMMs on hipBLASLt's default heuristics instead of the committed TunableOp "
                         "selections the model benchmarks load (before round 5's split-XCD runs the tool had no "
                         "TunableOp: its 'lib' rows were untuned)")
    args = ap.parse_args()
    if not args.untuned:
        from apex.utils.gemm_tuning import enable_tuned_gemms

        enable_tuned_gemms()
    M = args.M
    shapes = {}
    for item in args.shapes.split(","):
        name, nk = item.split(":")
        n, k = nk.split("x")
        shapes[name] = (int(n), int(k))
    torch.manual_seed(0)
    for name, (n, k) in shapes.items():
        dy = torch.randn(M, n, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(M, k, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(n, k, device="cuda", dtype=torch.bfloat16)
        paths = {"lib": "0"}
        for s in (int(x) for x in args.splits.split(",")):
            if M % 64 == 0 and M // 64 >= s:  # (slices of whole K-tiles, any count)
                paths[f"tt_s{s}"] = str(s)
        paths["auto"] = "auto"
        res = {p: [] for p in paths}
        outs = {}
        for p, v in paths.items():
            fused._WGRAD_TT = v
            fused._wgrad(dy, x, out=out)
            outs[p] = out.float().clone()
        for _ in range(5):
            for p, v in paths.items():
                fused._WGRAD_TT = v
                fused._wgrad(dy, x, out=out)
                torch.cuda.synchronize()
                e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                e[0].record()
                for _ in range(10):
                    fused._wgrad(dy, x, out=out)
                e[1].record()
                torch.cuda.synchronize()
                res[p].append(e[0].elapsed_time(e[1]) * 100.0)
        for p in paths:
            print(json.dumps({"shape": name, "M": M, "N": n, "K": k, "path": p, "us": round(statistics.median(res[p]), 1),
                              "max_abs_diff_vs_lib": float((outs[p] - outs["lib"]).abs().max())}), flush=True)
        fused._WGRAD_TT = "auto"
        del dy, x, out


if __name__ == "__main__":
    main()
