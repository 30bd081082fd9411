"""Own persistent MFMA GEMM (C.gemm) vs hipBLASLt (torch.mm / addmm with the committed TunableOp
selections) at the BERT-Large b768 plain / bias-only product shapes and 8192^3: time, board power,
clock and energy per call, on random bf16 operands.

  python tools/gemm_energy_vs_lib.py power [seconds]   # per (shape, impl): a back-to-back loop of
                                                       # `seconds`, amdsmi sampled every 50 ms;
                                                       # interleaved twice; one JSON line each
  python tools/gemm_energy_vs_lib.py run [reps]        # every (shape, impl) `reps` times (the body
                                                       # of the rocprofv3 --pmc passes,
                                                       # tools/gpu_gemm_pmc.sh)

Energy per call = mean board power x time per call (the whole board, idle floor included: compare
the two impls at equal work, not in absolute terms).
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (name, M, N, K, bias): the library keeps these in the BERT step (profiles/README.md round 5)
SHAPES = [("qkv_fwd_bias", 98304, 3072, 1024, True), ("attn_out_fwd", 98304, 1024, 1024, False),
          ("ffn2_fwd", 98304, 1024, 4096, False), ("sq8192", 8192, 8192, 8192, False)]


def _setup():
    from apex.utils.gemm_tuning import enable_tuned_gemms

    enable_tuned_gemms()
    import apex._ext as e

    return e.require()


def _fns(C, M, N, K, bias):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    w = (torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g) * K ** -0.5)
    b = torch.empty(N, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g) if bias else None
    if bias:
        return {"hipblaslt": lambda: torch.addmm(b, a, w.t()), "apex_persist": lambda: C.gemm(a, w, C.EPI_BIAS, b)}
    return {"hipblaslt": lambda: torch.mm(a, w.t()), "apex_persist": lambda: C.gemm(a, w, C.EPI_NONE)}


def power(seconds):
    from apex.utils.telemetry import GpuSampler

    C = _setup()
    for rnd in range(2):
        for name, M, N, K, bias in SHAPES:
            fns = _fns(C, M, N, K, bias)
            order = list(fns.items()) if rnd == 0 else list(fns.items())[::-1]
            for impl, f in order:
                for _ in range(3):
                    f()
                torch.cuda.synchronize()
                # warm the clock / power state for ~0.5 s before sampling
                t0 = time.time()
                while time.time() - t0 < 0.5:
                    f()
                torch.cuda.synchronize()
                smp = GpuSampler(period=0.05).start()
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                n = 0
                ev[0].record()
                t0 = time.time()
                while time.time() - t0 < seconds:
                    for _ in range(8):
                        f()
                    n += 8
                    if n % 64 == 0:
                        torch.cuda.synchronize()
                ev[1].record()
                torch.cuda.synchronize()
                s = smp.stop() or {}
                us = ev[0].elapsed_time(ev[1]) * 1000.0 / n
                pw = (s.get("power_w") or {}).get("mean")
                print(json.dumps({"round": rnd, "shape": name, "M": M, "N": N, "K": K, "impl": impl, "calls": n,
                                  "us_per_call": round(us, 2), "pflops": round(2.0 * M * N * K / us / 1e9, 3),
                                  "power_w_mean": pw, "sclk_mhz_mean": (s.get("sclk_mhz") or {}).get("mean"),
                                  "energy_mj_per_call": round(pw * us * 1e-3, 3) if pw else None,
                                  "tflop_per_joule": round(2.0 * M * N * K / (pw * us * 1e-6) / 1e12, 4) if pw else None}),
                      flush=True)
            del fns
            torch.cuda.empty_cache()


def run(reps):
    C = _setup()
    for name, M, N, K, bias in SHAPES:
        fns = _fns(C, M, N, K, bias)
        for impl, f in fns.items():
            for _ in range(reps):
                f()
            torch.cuda.synchronize()
            print(name, impl, "done", flush=True)
        del fns
        torch.cuda.empty_cache()


if __name__ == "__main__":
    mode = sys.argv[1] if len(sys.argv) > 1 else "power"
    if mode == "power":
        power(float(sys.argv[2]) if len(sys.argv) > 2 else 2.0)
    else:
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 3)
