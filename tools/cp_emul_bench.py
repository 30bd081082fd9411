"""Single-GPU emulation of context-parallel ring attention's compute (apex.transformer.context_parallel):
the block work of ALL W ranks of a zigzag ring (every visible (query chunk, key chunk) pair, the
log-sum-exp merges, the per-block backward and the dQ / dK / dV partial adds, in the partials'
transport dtype) run back to back on one GPU, against ONE flash-attention call over the full
sequence (forward + backward). The ratio is the compute overhead of splitting attention over the
ring; the P2P transfers overlap the blocks on real ranks and are not modelled.

  python tools/cp_emul_bench.py [--S 8192] [--W 4] [--H 20] [--D 128] [--B 1]
Prints one JSON line.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--S", type=int, default=8192)
    ap.add_argument("--W", type=int, default=4)
    ap.add_argument("--H", type=int, default=20)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--B", type=int, default=1)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    import apex
    from apex.contrib.multihead_attn.flash import flash_attention
    from apex.transformer import context_parallel as cp

    apex._ext.require()
    torch.manual_seed(0)
    B, S, H, D, W = a.B, a.S, a.H, a.D, a.W
    q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    do = torch.randn_like(q)
    scale = D ** -0.5

    def full():
        qq, kk, vv = (t.detach().requires_grad_() for t in (q, k, v))
        flash_attention(qq, kk, vv, causal=True, scale=scale).backward(do)

    n = 2 * W
    chunks = [t.chunk(n, dim=1) for t in (q, k, v, do)]

    def rank_shard(r, i):
        ids, _ = cp.chunk_ids(r, W, "zigzag")
        return torch.cat([chunks[i][j] for j in ids], dim=1).contiguous()

    local = [[rank_shard(r, i) for i in range(4)] for r in range(W)]

    def emul():
        # every rank's ring steps as apex.transformer.context_parallel runs them: one flash call per
        # step (_step_calls), the fused merges, the block backward and the partial adds
        for r in range(W):
            ql, _, _, dol = local[r]
            acc_o = acc_l = None
            aux = {}
            Sl = ql.shape[1]
            for step in range(W):
                src = (r - step) % W
                kl_, vl = local[src][1], local[src][2]
                for q_sel, k_sel, diag in cp._step_calls(r, src, W, "zigzag", True):
                    blocks = cp._step_fwd(cp._rows(ql, q_sel, 2, 1), cp._rows(kl_, k_sel, 2, 1),
                                          cp._rows(vl, k_sel, 2, 1), diag, scale, 0.0)
                    s0 = 0 if q_sel is None else q_sel * (Sl // 2)
                    for o, lse, _, _ in blocks:
                        acc_o, acc_l = cp._merge(acc_o, acc_l, o, lse, s0, Sl)
                    aux[(step, q_sel, k_sel)] = [(x, part) for _, _, x, part in blocks]
            out = acc_o.to(q.dtype)
            lse = acc_l
            dq = torch.zeros_like(ql, dtype=torch.float32)
            for step in range(W):
                src = (r - step) % W
                kl_, vl = local[src][1], local[src][2]
                dk_t = torch.zeros(kl_.shape, dtype=cp._dkv_transport_dtype(k), device=q.device)
                dv_t = torch.zeros_like(dk_t)
                for q_sel, k_sel, diag in cp._step_calls(r, src, W, "zigzag", True):
                    gs = cp._step_bwd(cp._rows(dol, q_sel, 2, 1), cp._rows(ql, q_sel, 2, 1), cp._rows(kl_, k_sel, 2, 1),
                                      cp._rows(vl, k_sel, 2, 1), cp._rows(out, q_sel, 2, 1), cp._rows(lse, q_sel, 2, 2),
                                      diag, scale, 0.0, aux[(step, q_sel, k_sel)])
                    for g in gs:
                        (dq if q_sel is None else dq.chunk(2, dim=1)[q_sel]).add_(g[0])
                        tk = dk_t if k_sel is None else dk_t.chunk(2, dim=1)[k_sel]
                        tv = dv_t if k_sel is None else dv_t.chunk(2, dim=1)[k_sel]
                        if g[3] is not None:
                            tk, tv = tk.chunk(2, dim=1)[g[3]], tv.chunk(2, dim=1)[g[3]]
                        tk.add_(g[1])
                        tv.add_(g[2])

    def bench(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record()
        for _ in range(a.iters):
            fn()
        e[1].record()
        torch.cuda.synchronize()
        return e[0].elapsed_time(e[1]) / a.iters

    t_full = bench(full)
    t_emul = bench(emul)
    print(json.dumps({"S": S, "W": W, "H": H, "D": D, "B": B, "full_flash_fwd_bwd_ms": round(t_full, 3),
                      "ring_all_ranks_ms": round(t_emul, 3), "overhead": round(t_emul / t_full - 1.0, 4),
                      "merge": "hip" if cp._native_merge(q, torch.empty(1, device=q.device)) else "torch",
                      "dkv_transport": str(cp._dkv_transport_dtype(k)).replace("torch.", ""),
                      "kv_split": os.environ.get("APEX_CP_KV_SPLIT", "0")}), flush=True)


if __name__ == "__main__":
    main()
