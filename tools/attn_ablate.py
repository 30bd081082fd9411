"""Attention backward ablation at one shape: time with parts of the kernel switched off through
AttnArgs.dbg (1 = no dQ section, 2 = no dV/dK products, 8 = no next-block prefetch) to see what the
kernel's time is made of. Diagnostics only (the outputs are wrong with any bit set).

Measured (profiles/r2_attn_bwd_ablation.jsonl, BERT b256 s128 h16 d64, p 0.1): 206 us full, 168
without dQ, 181 without the dK/dV products, 132 with dQ, dK/dV and the prefetch all off — the
kernel is a serial chain per workgroup (2 per CU at 237 VGPRs), not load-latency-bound: staging all
four query blocks up front (every load in flight at once) measured 201 vs 202 us and was dropped.

    python tools/attn_ablate.py [bert|gpt2|megatron] [p]
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.attn_bench import SHAPES, bench  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "bert"
    p = float(sys.argv[2]) if len(sys.argv) > 2 else 0.1
    import apex

    C = apex._ext.require()
    s = SHAPES[name]
    B, S, H, D, causal = s["B"], s["S"], s["H"], s["D"], s["causal"]
    qkv = torch.randn(B, S, 3, H, D, device="cuda", dtype=torch.bfloat16)
    q, k, v = qkv.unbind(2)
    scale = 1.0 / math.sqrt(D)
    o, lse, dmask = C.flash_attn_fwd(q, k, v, causal, scale, p, 1, 2, None)
    do = torch.randn_like(o)
    dqkv = torch.empty_like(qkv)
    dq, dk, dv = dqkv.unbind(2)
    dsum = torch.zeros(B, 3 * H * D, device="cuda")
    nbytes = 5 * q.numel() * 2 + 3 * q.numel() * 2
    t = bench(lambda: C.flash_attn_fwd(q, k, v, causal, scale, p, 1, 2, None))
    print(json.dumps({"shape": name, "p": p, "pass": "fwd", "us": round(t, 1),
                      "TBps": round(4 * q.numel() * 2 / t / 1e6, 2)}), flush=True)
    for dbg in (0, 1, 2, 8, 3, 11):
        t = bench(lambda: C.flash_attn_bwd(do, q, k, v, o, lse, dq, dk, dv, causal, scale, p, 1, 2, None, dmask,
                                           dsum, dbg))
        print(json.dumps({"shape": name, "p": p, "pass": "bwd+dsum", "dbg": dbg, "us": round(t, 1),
                          "TBps_if_full": round(nbytes / t / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
