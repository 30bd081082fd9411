"""LayerNorm backward kernel timing (the C op directly, CUDA events): python tools/ln_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import apex  # noqa: E402


def main():
    C = apex._ext.require()
    for rows, cols in ((8192, 2560), (8192, 4096), (98304, 1024), (16384, 1600)):
        x = torch.randn(rows, cols, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(cols, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(cols, device="cuda", dtype=torch.bfloat16)
        y, mean, rstd = C.ln_fwd(x, cols, w, b, 1e-5, False)
        dy = torch.randn_like(y)
        for _ in range(3):
            C.ln_bwd(dy, x, cols, w, b, mean, rstd, False, None, None)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            C.ln_bwd(dy, x, cols, w, b, mean, rstd, False, None, None)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"ln_bwd rows {rows} cols {cols}: {us:.1f} us  {3 * rows * cols * 2 / us / 1e6:.2f} TB/s (x, dy, dx)")


if __name__ == "__main__":
    main()
