"""BERT MLM decoder GEMMs at the bench shape (768 x 19 masked positions, hidden 1024) for the
vocab padded to 64 (30528, the model default) vs 256 (30720): forward logits (fused_dense with
bias), input gradient and weight gradient, as the training step runs them. One JSON line per
(vocab, op): us per call.

  python tools/mlm_head_bench.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters=20, warm=3):
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
    from apex.utils.gemm_tuning import enable_tuned_gemms

    enable_tuned_gemms()
    from apex.ops import fused as fops

    T, H = 768 * 19, 1024
    t = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
    for V in (30528, 30720):
        w = torch.randn(V, H, device="cuda", dtype=torch.bfloat16) * 0.02
        b = torch.zeros(V, device="cuda", dtype=torch.bfloat16)
        g = torch.randn(T, V, device="cuda", dtype=torch.bfloat16)
        ops = {
            "fwd": lambda: fops.fused_dense(t, w, b),
            "dgrad": lambda: torch.mm(g, w),
            "wgrad": lambda: fops._wgrad(g, t),
        }
        for name, fn in ops.items():
            us = timed(fn)
            print(json.dumps({"vocab": V, "op": name, "us": round(us, 1),
                              "pflops": round(2.0 * T * V * H / us / 1e9, 3)}), flush=True)


if __name__ == "__main__":
    main()
