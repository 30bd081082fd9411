"""Flash-attention microbenchmark (fwd / bwd separately) on the model shapes.

  python tools/attn_bench.py [--only bert|gpt2|megatron]

Prints one JSON line per (shape, dropout, pass) with time and achieved TFLOP/s
(causal FLOPs counted as half of the dense ones).
"""
import argparse
import json
import math

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {
    "bert": dict(B=256, S=128, H=16, D=64, causal=False),
    "bert768": dict(B=768, S=128, H=16, D=64, causal=False),
    "gpt2": dict(B=8, S=1024, H=25, D=64, causal=True),
    "megatron": dict(B=4, S=2048, H=20, D=128, causal=True),
}


def bench(fn, iters=10, warm=3):
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
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    import apex

    C = apex._ext.require()
    for name, s in SHAPES.items():
        if a.only and name != a.only:
            continue
        B, S, H, D, causal = s["B"], s["S"], s["H"], s["D"], s["causal"]
        qkv = torch.randn(B, S, 3, H, D, device="cuda", dtype=torch.bfloat16)
        q, k, v = qkv.unbind(2)
        flops = 4.0 * B * H * S * S * D * (0.5 if causal else 1.0)
        for p in (0.0, 0.1):
            scale = 1.0 / math.sqrt(D)
            o, lse, dmask = C.flash_attn_fwd(q, k, v, causal, scale, p, 1, 2, None)
            t_f = bench(lambda: C.flash_attn_fwd(q, k, v, causal, scale, p, 1, 2, None))
            do = torch.randn_like(o)
            dqkv = torch.empty_like(qkv)
            dq, dk, dv = dqkv.unbind(2)
            t_b = bench(lambda: C.flash_attn_bwd(do, q, k, v, o, lse, dq, dk, dv, causal, scale, p, 1, 2, None,
                                                 dmask))
            dsum = torch.zeros(B, 3 * H * D, device="cuda")
            t_bs = bench(lambda: C.flash_attn_bwd(do, q, k, v, o, lse, dq, dk, dv, causal, scale, p, 1, 2, None,
                                                  dmask, dsum))
            t_cs = bench(lambda: C.colsum(dqkv.view(B * S, 3 * H * D), torch.bfloat16))
            for pas, t, f in (("fwd", t_f, flops), ("bwd", t_b, 2.5 * flops), ("bwd+dsum", t_bs, 2.5 * flops),
                              ("separate colsum", t_cs, 0.0)):
                print(json.dumps({"shape": name, "p": p, "pass": pas, "us": round(t, 1),
                                  "tflops": round(f / t / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
