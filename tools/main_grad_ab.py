"""A/B of the fp32 main_grad accumulation paths on the Megatron GPT shapes (GPU box):
split-K fp32 slabs + splitk_reduce(accumulate) vs one addmm with out_dtype=fp32 and beta=1
accumulating straight into main_grad (hipBLASLt C = D = fp32) vs the transposed-read MFMA kernel
with the fp32 read-modify-write epilogue (C.gemm_tt_acc), vs the bf16 dW baseline (TunableOp
selections loaded as in the benches) alone and followed by the fp32 add into main_grad.

  python tools/main_grad_ab.py [tokens=8192] [hidden=2560]
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from apex.utils import gemm_tuning  # noqa: E402

gemm_tuning.enable_tuned_gemms()
from apex import _ext  # noqa: E402
from apex.ops import fused as F  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 2560
    C = _ext.require()
    for (N, K) in [(3 * H, H), (H, H), (4 * H, H), (H, 4 * H)]:
        dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        mg = torch.zeros(N, K, device="cuda", dtype=torch.float32)
        ref = dy.t().float() @ x.float()

        def slabs():
            s = F._wgrad_splits(M, N, K)
            sl = torch.bmm(dy.view(s, M // s, N).transpose(1, 2), x.view(s, M // s, K), out_dtype=torch.float32)
            C.splitk_reduce(sl, torch.float32, mg, accumulate=True)

        def addmm():
            torch.addmm(mg, dy.t(), x, out_dtype=torch.float32, out=mg)

        def bf16():
            torch.mm(dy.t(), x)

        def bf16_add():
            mg.add_(torch.mm(dy.t(), x))

        def tt_acc():
            C.gemm_tt_acc(dy, x, mg)

        row = {"M": M, "N": N, "K": K}
        for name, fn in (("slabs_reduce", slabs), ("addmm_fp32_beta1", addmm), ("tt_acc", tt_acc),
                         ("bf16_dW", bf16), ("bf16_dW_add", bf16_add)):
            try:
                mg.zero_()
                fn()
                torch.cuda.synchronize()
                err = float((mg - ref).abs().max() / ref.abs().max()) if name != "bf16_dW" else None
                row[name] = {"us": round(timeit(fn), 1), "rel_err": err}
            except Exception as e:  # noqa: BLE001
                row[name] = {"error": str(e)[:200]}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
