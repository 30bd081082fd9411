"""Plain NT products: hipBLASLt (torch.mm, the committed TunableOp selections) vs apex's MFMA GEMM
(C.gemm, EPI_NONE) on random bf16 at 8192^3 and the BERT-Large plain-product shapes (M = 98304).
Interleaved rounds in one process; prints one JSON line per (shape, impl): min / median us, PF/s.

  python tools/gemm_lib_ref.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from apex.utils.gemm_tuning import enable_tuned_gemms

    enable_tuned_gemms()
    import apex._ext as e

    C = e.require()
    shapes = [(8192, 8192, 8192), (98304, 3072, 1024), (98304, 1024, 1024), (98304, 1024, 4096),
              (98304, 4096, 1024)]
    for M, N, K in shapes:
        a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1) * K ** -0.5
        fns = {"hipblaslt": lambda: torch.mm(a, b.t()), "apex_mfma": lambda: C.gemm(a, b, 0)}
        ts = {k: [] for k in fns}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for _ in range(5):
            for k, f in fns.items():
                f()
                ev[0].record()
                for _ in range(5):
                    f()
                ev[1].record()
                torch.cuda.synchronize()
                ts[k].append(ev[0].elapsed_time(ev[1]) / 5 * 1000)
        for k, t in ts.items():
            t.sort()
            print(json.dumps({"M": M, "N": N, "K": K, "impl": k, "us_min": round(t[0], 1), "us_med": round(t[2], 1),
                              "pflops": round(2.0 * M * N * K / t[0] / 1e9, 3)}), flush=True)
        del a, b


if __name__ == "__main__":
    main()
