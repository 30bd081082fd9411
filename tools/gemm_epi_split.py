"""Split the FFN1 forward GEMM (bias + GELU + stored derivative epilogue, M = 98304, N = 4096,
K = 1024) into its parts with a diagnostics build (g_gemm_dbg): 0 full, 2 no epilogue,
3 epilogue without the GELU math (stores kept), 4 GELU math without the stores."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.gemm_mfma_bench import bench  # noqa: E402


def main():
    import apex._ext as e
    C = e.require()
    M = int(os.environ.get("PB_M", 98304))
    x = torch.empty(M, 1024, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    w = torch.empty(4096, 1024, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1) * 0.03
    b = torch.empty(4096, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    g = torch.empty(M, 4096, device="cuda", dtype=torch.bfloat16)
    res = {}
    for _ in range(3):
        for dbg in (0, 2, 3, 4):
            C.gemm_set_dbg(dbg)
            t = bench(lambda: C.gemm(x, w, 8, b))
            res[dbg] = min(res.get(dbg, 1e30), t)
        C.gemm_set_dbg(0)
        t = bench(lambda: torch.mm(x, w.t(), out=g))
        res["lib_mm"] = min(res.get("lib_mm", 1e30), t)
    print(json.dumps({"M": M, **{str(k): round(v, 1) for k, v in res.items()}}))


if __name__ == "__main__":
    main()
