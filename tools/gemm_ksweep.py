"""Fixed-cost vs per-K-tile cost of the MFMA GEMM: time at M=32768, N=1024 over K (random bf16),
alongside torch.mm. A linear fit t(K) = a + b*K/64 separates prologue/epilogue from the main loop."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.gemm_mfma_bench import bench  # noqa: E402


def main():
    import apex._ext as e

    C = e.require()
    M = int(os.environ.get("KS_M", 32768))
    for N in (1024, 4096):
        for K in (64, 256, 1024, 4096):
            x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
            w = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
            r = {}
            for _ in range(3):
                for name, fn in (("torch.mm", lambda: torch.mm(x, w.t())), ("mfma", lambda: C.gemm(x, w, 0))):
                    r[name] = min(r.get(name, 1e30), bench(fn))
            print(json.dumps({"M": M, "N": N, "K": K, **{k: round(v, 1) for k, v in r.items()}}), flush=True)


if __name__ == "__main__":
    main()
