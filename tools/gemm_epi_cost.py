"""Epilogue cost of the MFMA GEMM: full kernel vs main loop only (g_gemm_dbg = 2) on the
BERT-Large FFN shapes (M = 32768). Prints JSON lines."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.attn_bench import bench  # noqa: E402


def main():
    import apex._ext as e

    C = e.require()
    for (M, N, K, epi) in ((32768, 4096, 1024, 0), (32768, 4096, 1024, 2), (32768, 4096, 1024, 8),
                          (32768, 4096, 1024, 3), (32768, 4096, 1024, 10), (32768, 1024, 4096, 0),
                          (32768, 1024, 3072, 4), (32768, 1024, 1024, 0)):
        x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        w = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
        aux = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)

        def run():
            if epi == 0:
                C.gemm(x, w, 0)
            elif epi in (1, 2, 8, 9):
                C.gemm(x, w, epi, b)
            else:
                C.gemm(x, w, epi, None, aux, torch.bfloat16 if epi in (3, 10) else None)
        res = {"M": M, "N": N, "K": K, "epi": epi}
        for dbg in (0, 2):
            C.gemm_set_dbg(dbg)
            res[f"dbg{dbg}_us"] = round(bench(run, iters=20), 1)
        C.gemm_set_dbg(0)
        res["lib_mm_us"] = round(bench(lambda: torch.mm(x, w.t()), iters=20), 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
