"""fp32 attention: the f32-MFMA flash kernels (csrc/attention_f32.hip) vs the torch compositions
they replace (the dense fused-softmax composition at training lengths, the query-blocked one
beyond), forward + backward through the same autograd entry the models use.

  python tools/attn_f32_bench.py [--only bert|gpt2|megatron]

One JSON line per (shape, dropout, path): ms per forward+backward and the f32 MFMA TFLOP/s it
implies (fwd 4 B H S^2 D, bwd 2.5x that; causal halves both; the f32 matrix peak is ~157 TF).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {
    "bert": dict(B=256, S=128, H=16, D=64, causal=False),  # the bench's fp32 micro-batch
    "gpt2": dict(B=8, S=1024, H=25, D=64, causal=True),
    "megatron": dict(B=4, S=2048, H=20, D=128, causal=True),
}


def timed(fn, iters=5, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(iters):
        fn()
    e[1].record()
    torch.cuda.synchronize()
    return e[0].elapsed_time(e[1]) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    from apex.contrib.multihead_attn import attention as att

    for name, s in SHAPES.items():
        if a.only and name != a.only:
            continue
        B, S, H, D, causal = s["B"], s["S"], s["H"], s["D"], s["causal"]
        q, k, v = (torch.randn(B, S, H, D, device="cuda", requires_grad=True) for _ in range(3))
        do = torch.randn(B, S, H, D, device="cuda")
        flops = 3.5 * 4.0 * B * H * S * S * D * (0.5 if causal else 1.0)
        for p in (0.0, 0.1):
            for path in ("kernel", "composition"):
                os.environ["APEX_ATTN_F32"] = "1" if path == "kernel" else "0"

                def step():
                    o = att.attention(q, k, v, dropout_p=p, causal=causal)
                    torch.autograd.backward(o, do)

                torch.cuda.reset_peak_memory_stats()
                base = torch.cuda.memory_allocated()
                ms = timed(step)
                peak = (torch.cuda.max_memory_allocated() - base) / 2 ** 20
                print(json.dumps({"shape": name, "B": B, "S": S, "H": H, "D": D, "causal": causal, "p": p,
                                  "path": path, "ms_fwd_bwd": round(ms, 3), "tflops": round(flops / ms / 1e9, 1),
                                  "peak_extra_mib": round(peak, 1)}), flush=True)
        os.environ.pop("APEX_ATTN_F32", None)


if __name__ == "__main__":
    main()
