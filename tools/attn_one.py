"""One attention shape, fwd or bwd only, N launches (for rocprofv3 --pmc passes).

  python tools/attn_one.py bert|gpt2|megatron fwd|bwd [p] [iters]
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.attn_bench import SHAPES  # noqa: E402


def main():
    name, pas = sys.argv[1], sys.argv[2]
    p = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10
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
    for _ in range(iters):
        if pas == "fwd":
            C.flash_attn_fwd(q, k, v, causal, scale, p, 1, 2, None)
        else:
            C.flash_attn_bwd(do, q, k, v, o, lse, dq, dk, dv, causal, scale, p, 1, 2, None, dmask)
    torch.cuda.synchronize()
    print("ok", name, pas)


if __name__ == "__main__":
    main()
