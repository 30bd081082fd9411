"""Bandwidth of the BERT bias+dropout+residual+LayerNorm kernels against plain streams of the same
shape (98304 x 1024 bf16): torch copy (1 read + 1 write), torch add (2 + 1), the LN forward
(t, residual -> y: 2 + 1) and the memory-efficient backward (dy, y -> dres, dt: 2 + 2). CUDA events,
median of 5 rounds of 20 calls; TB/s over the tensor bytes each op must move.

    python tools/bdaln_bw_probe.py > profiles/r6_bdaln_bw_probe.jsonl
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, rounds=5):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(rounds):
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
    M, E = 98304, 1024
    dt = torch.bfloat16
    nb = M * E * 2
    a = torch.randn(M, E, device="cuda", dtype=dt)
    b = torch.randn(M, E, device="cuda", dtype=dt)
    c = torch.empty_like(a)
    bias = torch.randn(E, device="cuda", dtype=dt)
    gamma = (torch.rand(E, device="cuda") + 0.5).to(dt)
    beta = torch.randn(E, device="cuda", dtype=dt)

    def rec(name, us, tensors):
        print(json.dumps(dict(op=name, us=round(us, 1), tb_s=round(tensors * nb / us / 1e6, 2))), flush=True)

    rec("copy", timeit(lambda: c.copy_(a)), 2)
    rec("add", timeit(lambda: torch.add(a, b, out=c)), 3)
    y, s, mean, rstd = C.bdaln_fwd(a, bias, b, gamma, beta, 1e-12, 0.1, 3, 4, store_s=False, s_cond=True)
    rec("bdaln_fwd_p0.1", timeit(lambda: C.bdaln_fwd(a, bias, b, gamma, beta, 1e-12, 0.1, 3, 4, store_s=False,
                                                        s_cond=True)), 3)
    rec("bdaln_fwd_p0", timeit(lambda: C.bdaln_fwd(a, bias, b, gamma, beta, 1e-12, 0.0, 3, 4, store_s=False,
                                                      s_cond=True)), 3)
    dy = torch.randn_like(a)
    dg, db, dbo = (torch.empty(E, device="cuda", dtype=dt) for _ in range(3))
    rec("bdaln_bwd_p0.1", timeit(lambda: C.bdaln_bwd(dy, y, gamma, mean, rstd, 0.1, 3, 4, True, dgamma_out=dg,
                                                        dbeta_out=db, dbias_out=dbo, beta=beta)), 4)
    rec("bdaln_bwd_p0", timeit(lambda: C.bdaln_bwd(dy, y, gamma, mean, rstd, 0.0, 3, 4, True, dgamma_out=dg,
                                                      dbeta_out=db, dbias_out=dbo, beta=beta)), 4)


if __name__ == "__main__":
    main()
