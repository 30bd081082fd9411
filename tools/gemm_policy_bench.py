"""Library GEMM (+ separate HIP epilogue kernels) vs the MFMA GEMM with the epilogue fused, for
every dense GEMM of a BERT-Large layer at M = 32768 tokens (random bf16). Decides the per-call
policy in apex/ops/gemm.py. Interleaved rounds in one process; us per call.

  python tools/gemm_policy_bench.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.gemm_mfma_bench import bench  # noqa: E402


def r(*s):
    return torch.empty(*s, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)


def main():
    from apex.utils.gemm_tuning import enable_tuned_gemms

    enable_tuned_gemms()  # the same committed library selections the benchmark loads
    import apex._ext as e
    from apex.ops.fused import _wgrad

    from apex.ops import fused

    fused._WGRAD_TT = "0"  # "lib" below = the library split-K path
    C = e.require()
    M = int(os.environ.get("PB_M", 32768))
    H, F = 1024, 4096
    x, g, o = r(M, H), r(M, F), r(M, H)
    wqkv, wo, w1, w2 = r(3 * H, H) * 0.03, r(H, H) * 0.03, r(F, H) * 0.03, r(H, F) * 0.03
    bqkv, b1 = r(3 * H), r(F)
    dt, dqkv, dh, h, dres = r(M, H), r(M, 3 * H), r(M, F), r(M, F), r(M, H)
    wqkvT, woT, w1T, w2T = (C.transpose(w) for w in (wqkv, wo, w1, w2))
    cases = {
        "qkv_fwd": {"lib": lambda: torch.addmm(bqkv, x, wqkv.t()), "mfma": lambda: C.gemm(x, wqkv, 1, bqkv)},
        "attn_out_fwd": {"lib": lambda: torch.mm(o, wo.t()), "mfma": lambda: C.gemm(o, wo, 0)},
        "ffn1_fwd": {"lib": lambda: C.bias_act_fwd(torch.mm(x, w1.t()), b1, 0),
                     "mfma": lambda: C.gemm(x, w1, 2, b1)},
        "ffn2_fwd": {"lib": lambda: torch.mm(g, w2.t()), "mfma": lambda: C.gemm(g, w2, 0)},
        "attn_out_dgrad": {"lib": lambda: torch.mm(dt, wo), "mfma": lambda: C.gemm(dt, woT, 0)},
        "qkv_dgrad_resid": {"lib": lambda: torch.addmm(dres, dqkv, wqkv), "mfma": lambda: C.gemm(dqkv, wqkvT, 4, None, dres),
                            "lib_mm_add": lambda: torch.mm(dqkv, wqkv).add_(dres)},
        "ffn2_dgrad_dgelu": {"lib": lambda: C.bias_act_bwd(torch.mm(dt, w2), h, None, 0)[0],
                             "mfma": lambda: C.gemm(dt, w2T, 3, None, h, torch.bfloat16)},
        "ffn1_dgrad_resid": {"lib": lambda: torch.addmm(dres, dh, w1), "mfma": lambda: C.gemm(dh, w1T, 4, None, dres),
                             "lib_mm_add": lambda: torch.mm(dh, w1).add_(dres)},
        "transpose_w1": {"mfma": lambda: C.transpose(w1)},
        "wgrad_qkv": {"lib": lambda: _wgrad(dqkv, x), "mfma_s2": lambda: C.gemm_tt(dqkv, x, 2, torch.bfloat16),
                      "mfma_s4": lambda: C.gemm_tt(dqkv, x, 4, torch.bfloat16)},
        "wgrad_o": {"lib": lambda: _wgrad(dt, o), "mfma_s4": lambda: C.gemm_tt(dt, o, 4, torch.bfloat16),
                    "mfma_s8": lambda: C.gemm_tt(dt, o, 8, torch.bfloat16),
                    "mfma_s16": lambda: C.gemm_tt(dt, o, 16, torch.bfloat16)},
        "wgrad_1": {"lib": lambda: _wgrad(dh, x), "mfma_s2": lambda: C.gemm_tt(dh, x, 2, torch.bfloat16),
                    "mfma_s4": lambda: C.gemm_tt(dh, x, 4, torch.bfloat16)},
        "wgrad_2": {"lib": lambda: _wgrad(dt, g), "mfma_s2": lambda: C.gemm_tt(dt, g, 2, torch.bfloat16),
                    "mfma_s4": lambda: C.gemm_tt(dt, g, 4, torch.bfloat16)},
    }
    for name, vs in cases.items():
        best = {k: 1e30 for k in vs}
        for _ in range(3):
            for k, fn in vs.items():
                best[k] = min(best[k], bench(fn))
        print(json.dumps({"case": name, **{k: round(v, 1) for k, v in best.items()}}), flush=True)


if __name__ == "__main__":
    main()
