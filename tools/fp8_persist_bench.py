"""fp8 GEMMs of the BERT-Large fp8 step at M = 98304 tokens, per epilogue, on whichever kernel
this process's APEX_GEMM_PERSIST_F8 selects (1: persistent, 0: one tile per workgroup). Run it
twice to A/B (the switch is read once per process):

    APEX_GEMM_PERSIST_F8=1 python tools/fp8_persist_bench.py >> out.jsonl
    APEX_GEMM_PERSIST_F8=0 python tools/fp8_persist_bench.py >> out.jsonl

One JSON line per shape: us per call (median of 5 rounds of 10), PF/s, and a checksum of the
output (equal across the two runs: the kernels are bitwise identical by construction).
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import apex._ext as e

    C = e.require()
    M = int(os.environ.get("M", 98304))
    mode = os.environ.get("APEX_GEMM_PERSIST_F8", "1")
    one = torch.ones(1, device="cuda")
    torch.manual_seed(0)
    shapes = [("qkv_fwd_bias", 3072, 1024, "EPI_BIAS", 0, False), ("attn_out_fwd", 1024, 1024, "EPI_NONE", 0, False),
              ("ffn1_fwd_gelu_d_q8", 4096, 1024, "EPI_BIAS_GELU_D", 0, True),
              ("ffn2_fwd", 1024, 4096, "EPI_NONE", 0, False), ("ffn2_dgrad_mul_q8", 4096, 1024, "EPI_MUL", 1, True),
              ("ffn1_dgrad_resid", 1024, 4096, "EPI_RESID", 1, False)]
    for name, N, K, epi_name, fmt_a, q8 in shapes:
        a8 = C.fp8_quantize(torch.randn(M, K, device="cuda").bfloat16(), fmt_a, one * 4)
        w8 = C.fp8_quantize((torch.randn(N, K, device="cuda") * 0.05).bfloat16(), 0, one * 100)
        ia, iw = one / 4, one / 100
        epi = getattr(C, epi_name)
        bias = (torch.randn(N, device="cuda") * 0.1).bfloat16() if epi_name in ("EPI_BIAS", "EPI_BIAS_GELU_D") else None
        aux = torch.randn(M, N, device="cuda").bfloat16() if epi_name in ("EPI_MUL", "EPI_RESID") else None
        bgd = torch.float32 if epi_name == "EPI_MUL" else None
        kw = {}
        if q8:
            kw = dict(q8_out=torch.empty(M, N, dtype=torch.uint8, device="cuda"), q8_scale=one * 2,
                      q8_amax=torch.zeros(1, device="cuda"), q8_fmt=fmt_a)

        def f():
            return C.gemm_f8(a8, w8, ia, iw, fmt_a, epi, bias, aux, bgd, torch.bfloat16, **kw)

        out = f()
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(10):
                f()
            ev[1].record()
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]) * 100.0)
        us = statistics.median(ts)
        chk = float(out[0].float().sum())
        if q8:
            chk += float(kw["q8_out"].float().sum()) * 1e-6
        print(json.dumps({"shape": name, "persistent": mode != "0", "M": M, "N": N, "K": K, "epi": epi_name, "q8": q8,
                          "us": round(us, 1), "pflops": round(2.0 * M * N * K / us / 1e9, 3),
                          "checksum": chk}), flush=True)
        del a8, w8, aux, out, kw


if __name__ == "__main__":
    main()
