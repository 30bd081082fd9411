"""Attention backward section costs: time the backward with diagnostic skip bits (csrc
AttnArgs::dbg: 1 = no dQ section, 2 = no dV/dK products, 8 = no global prefetch in the loop).
Results are numerically meaningless; only the timings are."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.attn_bench import SHAPES, bench  # noqa: E402


def main():
    import apex

    C = apex._ext.require()
    for name in ("bert", "gpt2"):
        s = SHAPES[name]
        B, S, H, D, causal = s["B"], s["S"], s["H"], s["D"], s["causal"]
        qkv = torch.randn(B, S, 3, H, D, device="cuda", dtype=torch.bfloat16)
        q, k, v = qkv.unbind(2)
        scale = 1.0 / math.sqrt(D)
        p = 0.1
        o, lse, dmask = C.flash_attn_fwd(q, k, v, causal, scale, p, 1, 2, None)
        do = torch.randn_like(o)
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = dqkv.unbind(2)
        for dbg in (0, 1, 2, 3, 8, 11):
            t = bench(lambda: C.flash_attn_bwd(do, q, k, v, o, lse, dq, dk, dv, causal, scale, p, 1, 2, None, dmask,
                                               None, dbg), iters=20)
            print(json.dumps({"shape": name, "dbg": dbg, "us": round(t, 1)}), flush=True)


if __name__ == "__main__":
    main()
