"""Where do a fused GEMM epilogue's outputs differ from the fp32 reference? Prints, per output,
the max error and the distinct (row % 256, col % 256) blocks of the bad elements."""
import sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import apex._ext as e

C = e.require()
torch.manual_seed(0)
M, N, K = 4096, 4096, 1024
a = torch.randn(M, K, device="cuda").bfloat16()
b = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
bias = torch.randn(N, device="cuda").bfloat16()
ref = a.float() @ b.float().t() + bias.float()
for epi in (1, 2, 8):
    y, h = C.gemm(a, b, epi, bias)
    outs = {"y": y} if epi == 1 else {"y": y, "aux": h}
    for name, t in outs.items():
        r = ref if (epi == 1 or name == "aux" and epi == 2) else None
        if r is None:
            g = torch.nn.functional.gelu(ref.bfloat16().float())
            r = g if name == "y" else None
        if r is None:
            continue
        err = (t.float() - r).abs()
        bad = err > 0.05 * r.abs().max()
        idx = bad.nonzero()
        print(epi, name, "maxerr", float(err.max()), "nbad", int(bad.sum()), flush=True)
        if idx.numel():
            rows = sorted(set((idx[:, 0] % 256).tolist()))
            cols = sorted(set((idx[:, 1] % 256).tolist()))
            print("  rows%256", rows[:40], len(rows), "cols%256", cols[:40], len(cols))
            print("  tiles", sorted(set(((idx[:, 0] // 256) * 100 + idx[:, 1] // 256).tolist()))[:20])
