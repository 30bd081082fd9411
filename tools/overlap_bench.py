"""Does running the weight-gradient GEMMs on a side stream, concurrently with the input-gradient
chain, shorten one BERT-Large layer's backward on MI355X?

The input-gradient chain of a layer (bdaln bwd -> FFN2 dgrad x gelu' -> FFN1 dgrad + residual ->
bdaln bwd -> attn-out dgrad -> flash attention bwd -> QKV dgrad + residual) has long phases where
the matrix cores idle: the bandwidth-bound GEMM epilogues, the LayerNorm backward kernels and the
short-sequence attention backward. The four weight-gradient GEMMs do not feed that chain, so they
can fill those gaps if they run on another stream.

Interleaved rounds in one process, us per layer backward; M = tokens (default 98304 = b768 s128).

  python tools/overlap_bench.py [--m 98304] [--rounds 5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=98304)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from apex.utils.gemm_tuning import enable_tuned_gemms

    enable_tuned_gemms()
    import apex._ext as e
    from apex.ops import gemm as G
    from apex.ops.fused import _wgrad

    C = e.require()
    M, H, F, heads, S = a.m, 1024, 4096, 16, 128
    B = M // S

    def r(*s, scale=1.0):
        return (torch.empty(*s, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1) * scale)

    x, o, g, gd, dy = r(M, H), r(M, H), r(M, F), r(M, F), r(M, H)
    s_ln, gamma = r(M, H), r(H) + 1.0
    mean, rstd = torch.zeros(M, device="cuda"), torch.ones(M, device="cuda")
    wqkv, wo, w1, w2 = r(3 * H, H, scale=0.03), r(H, H, scale=0.03), r(F, H, scale=0.03), r(H, F, scale=0.03)
    qkv = r(B, S, 3, heads, H // heads)
    att_o = r(B, S, heads, H // heads)
    lse = torch.zeros(B, heads, S, device="cuda")
    grads = {}

    def chain(side):
        """one layer's backward; side = None (one stream) or a torch.cuda.Stream for the wgrads"""
        cur = torch.cuda.current_stream()

        def wg(name, dy_, x_):
            if side is None:
                grads[name] = _wgrad(dy_, x_)
                return
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                grads[name] = _wgrad(dy_, x_)
            dy_.record_stream(side)
            x_.record_stream(side)

        # FFN sublayer backward
        dres, dt, _, _, _ = C.bdaln_bwd(dy, s_ln, gamma, mean, rstd, 0.1, 1, 2, True)
        dh, _ = G.dgrad_mul(dt, w2, gd, torch.bfloat16)
        wg("w2", dt, g)
        dx1 = G.dgrad_resid(dh, w1, dres)
        wg("w1", dh, x)
        # attention sublayer backward
        dres2, dt2, _, _, _ = C.bdaln_bwd(dx1, s_ln, gamma, mean, rstd, 0.1, 3, 4, True)
        dctx = G.dgrad(dt2, wo).view(B, S, heads, H // heads)
        wg("wo", dt2, o)
        q, k, v = qkv.unbind(2)
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = dqkv.unbind(2)
        C.flash_attn_bwd(dctx, q, k, v, att_o, lse, dq, dk, dv, False, 0.125, 0.0, 0, 0, None, None, None)
        d2 = dqkv.view(M, 3 * H)
        dx = G.dgrad_resid(d2, wqkv, dres2)
        wg("wqkv", d2, x)
        if side is not None:
            cur.wait_stream(side)
        return dx

    side = torch.cuda.Stream()
    variants = {"one_stream": lambda: chain(None), "wgrad_side_stream": lambda: chain(side)}
    for fn in variants.values():
        for _ in range(2):
            fn()
    torch.cuda.synchronize()
    res = {k: [] for k in variants}
    for _ in range(a.rounds):
        for k, fn in variants.items():
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(a.iters):
                fn()
            ev[1].record()
            torch.cuda.synchronize()
            res[k].append(ev[0].elapsed_time(ev[1]) / a.iters * 1000.0)
    out = {k: {"min_us": round(min(v), 1), "median_us": round(sorted(v)[len(v) // 2], 1)} for k, v in res.items()}
    out["M"] = M
    print(json.dumps(out))


if __name__ == "__main__":
    main()
