"""Run one GEMM configuration N times (for rocprofv3 counter passes).
  python tools/gemm_one.py M N K [unused] [epi] [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import apex._ext as e

    C = e.require()
    M, N, K = (int(v) for v in sys.argv[1:4])
    epi = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    iters = int(sys.argv[6]) if len(sys.argv) > 6 else 20
    x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    w = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    aux = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(iters):
        if epi < 0:
            torch.mm(x, w.t())
        elif epi == 0:
            C.gemm(x, w, 0)
        elif epi in (1, 2):
            C.gemm(x, w, epi, b)
        else:
            C.gemm(x, w, epi, None, aux, torch.bfloat16 if epi == 3 else None)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
