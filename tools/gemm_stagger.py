"""Experiment: first-round stagger of the MFMA GEMM (g_gemm_stagger; st100 = none) vs epilogue cost."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.attn_bench import bench  # noqa: E402


def main():
    import apex._ext as e

    C = e.require()
    for (M, N, K, epi) in ((32768, 4096, 1024, 2), (32768, 4096, 1024, 3), (32768, 1024, 3072, 4),
                          (32768, 1024, 4096, 4), (32768, 4096, 1024, 0)):
        x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        w = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
        aux = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)

        def run():
            if epi == 0:
                C.gemm(x, w, 0)
            elif epi in (1, 2):
                C.gemm(x, w, epi, b)
            else:
                C.gemm(x, w, epi, None, aux, torch.bfloat16 if epi == 3 else None)
        res = {"M": M, "N": N, "K": K, "epi": epi}
        run()
        for st in (100, 1, 2, 3):  # 100 = none
            C.gemm_set_dbg(-st)
            res[f"st{st}_us"] = round(bench(run, iters=30), 1)
        C.gemm_set_dbg(-200)  # back to the launcher's default
        res["default_us"] = round(bench(run, iters=30), 1)
        C.gemm_set_dbg(2)
        res["mainloop_us"] = round(bench(run, iters=30), 1)
        C.gemm_set_dbg(0)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
