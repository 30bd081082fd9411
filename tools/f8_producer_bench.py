"""What the fp8 producer-side codes cost inside their producer kernels, at BERT-Large b768
(98304 tokens, hidden 1024, 16 heads, p = 0.1): the flash forward (codes of O), the flash
backward (codes of dQ / dK / dV), and the bias+dropout+residual+LayerNorm forward / backward
(codes of y / dt). Per kernel, same process, interleaved rounds:
  off     no codes (the bf16 step's call)
  codes   codes + running amax from 0 (the fp8 step's call: a few blocks raise amax by atomics)
  noatom  codes, amax preset to 3e38 (every block's filter read sees a larger value: no atomics)
  fresh   codes with amax zeroed before EVERY call, as in the model (each producer slot starts
          the step at 0), minus the time of the zeroing alone
and, for reference, the standalone quantise pass (C.fp8_quantize) over the same output.

    python tools/f8_producer_bench.py > profiles/r5_f8_producer_cost.jsonl
"""
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reset=None, iters=10, rounds=5):
    out = []
    for _ in range(rounds):
        if reset:
            reset()
        fn()
        torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record()
        for _ in range(iters):
            fn()
        e[1].record()
        torch.cuda.synchronize()
        out.append(e[0].elapsed_time(e[1]) * 1000.0 / iters)
    return statistics.median(out)


def main():
    from apex import _ext

    C = _ext.require()
    dev = "cuda"
    B, S, H, D = 768, 128, 16, 64
    E = H * D
    M = B * S
    torch.manual_seed(0)
    scale = torch.full((1,), 8.0, device=dev)
    amax = torch.zeros(1, device=dev)
    rows = []

    def rec(kernel, variant, us):
        rows.append(dict(kernel=kernel, variant=variant, us=round(us, 1)))
        print(json.dumps(rows[-1]), flush=True)

    def variants(kernel, call, out_like):
        codes = torch.empty(out_like.numel(), dtype=torch.uint8, device=dev)
        res = {}
        for _ in range(2):  # interleave
            res.setdefault("off", []).append(timeit(lambda: call(None)))
            res.setdefault("codes", []).append(timeit(lambda: call(codes), reset=lambda: amax.zero_()))
            res.setdefault("noatom", []).append(timeit(lambda: call(codes), reset=lambda: amax.fill_(3e38)))
            zt = timeit(lambda: amax.zero_())
            res.setdefault("fresh", []).append(timeit(lambda: (amax.zero_(), call(codes))) - zt)
            res.setdefault("standalone_quantize", []).append(
                timeit(lambda: C.fp8_quantize(out_like, 0, scale, amax), reset=lambda: amax.zero_()))
        for k, v in res.items():
            rec(kernel, k, min(v))

    # ---- flash forward (codes of O, e4m3)
    qkv = torch.randn(B, S, 3, H, D, device=dev, dtype=torch.bfloat16)
    q, k, v = qkv.unbind(2)
    sm = 1.0 / math.sqrt(D)
    o, lse, dmask = C.flash_attn_fwd(q, k, v, False, sm, 0.1, 1, 2, None)

    def fwd(codes):
        kw = {} if codes is None else dict(q8_out=codes.view(B, S, H, D), q8_scale=scale, q8_amax=amax, q8_fmt=0)
        C.flash_attn_fwd(q, k, v, False, sm, 0.1, 1, 2, None, **kw)

    variants("attn_fwd", fwd, o)
    # ---- flash backward (codes of dQ, dK, dV, e5m2)
    do = torch.randn_like(o)
    dqkv = torch.empty_like(qkv)
    dq, dk, dv = dqkv.unbind(2)

    def bwd(codes):
        kw = {}
        if codes is not None:
            cq, ck, cv = codes[: dqkv.numel()].view(B, S, 3, H, D).unbind(2)
            kw = dict(q8_dq=cq, q8_dk=ck, q8_dv=cv, q8_scale=scale, q8_amax=amax, q8_fmt=1)
        C.flash_attn_bwd(do, q, k, v, o, lse, dq, dk, dv, False, sm, 0.1, 1, 2, None, dmask, None, **kw)

    variants("attn_bwd", bwd, dqkv)
    # ---- bias+dropout+residual+LayerNorm forward (codes of y, e4m3), memory-efficient mode
    t = torch.randn(M, E, device=dev, dtype=torch.bfloat16)
    x = torch.randn(M, E, device=dev, dtype=torch.bfloat16)
    bo = torch.randn(E, device=dev, dtype=torch.bfloat16)
    gamma = torch.rand(E, device=dev, dtype=torch.bfloat16) + 0.5
    beta = torch.randn(E, device=dev, dtype=torch.bfloat16)
    y, s, mean, rstd = C.bdaln_fwd(t, bo, x, gamma, beta, 1e-12, 0.1, 3, 4, store_s=False, s_cond=True)

    def lnf(codes):
        kw = {} if codes is None else dict(q8_out=codes.view(M, E), q8_scale=scale, q8_amax=amax, q8_fmt=0)
        C.bdaln_fwd(t, bo, x, gamma, beta, 1e-12, 0.1, 3, 4, store_s=False, s_cond=True, **kw)

    variants("bdaln_fwd", lnf, y)
    # ---- its backward (codes of dt, e5m2), rebuilding x-hat from y
    dy = torch.randn(M, E, device=dev, dtype=torch.bfloat16)
    dg = torch.empty(E, device=dev, dtype=torch.bfloat16)
    db = torch.empty(E, device=dev, dtype=torch.bfloat16)
    dbo = torch.empty(E, device=dev, dtype=torch.bfloat16)

    def lnb(codes):
        kw = {} if codes is None else dict(q8_out=codes.view(M, E), q8_scale=scale, q8_amax=amax, q8_fmt=1)
        C.bdaln_bwd(dy, y, gamma, mean, rstd, 0.1, 3, 4, True, dgamma_out=dg, dbeta_out=db, dbias_out=dbo,
                    beta=beta, **kw)

    variants("bdaln_bwd", lnb, y)


if __name__ == "__main__":
    main()
