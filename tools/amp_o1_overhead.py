"""Host-side cost of the legacy O1 cast engine (amp.init: Python cast wrappers patched onto torch
functions / Tensor methods) per op call, against plain torch and torch.autocast.

Each configuration runs in its own subprocess (amp.init patches process-wide). Small CPU tensors,
so the time is the dispatch path, not the math:   python tools/amp_o1_overhead.py [--device cuda]
"""
import argparse
import json
import subprocess
import sys
import time

CASES = {
    "F.linear": "F.linear(x, w, b)",
    "torch.mm": "torch.mm(x, w)",
    "torch.add (promote)": "torch.add(x, y)",
    "torch.cat (sequence)": "torch.cat([x, y], 0)",
    "x.float() (untouched)": "x.float()",
    "F.softmax (fp32 list)": "F.softmax(x, -1)",
}


def run(mode, device, n):
    import torch
    import torch.nn.functional as F  # noqa: F401

    sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
    if mode == "amp_o1":
        from apex import amp

        amp.init(enabled=True, half_dtype=torch.bfloat16)
    x = torch.randn(16, 16, device=device)
    y = torch.randn(16, 16, device=device)
    w = torch.randn(16, 16, device=device)
    b = torch.randn(16, device=device)
    env = {"torch": torch, "F": torch.nn.functional, "x": x, "y": y, "w": w, "b": b}
    out = {}
    for name, expr in CASES.items():
        code = compile(expr, name, "eval")
        ctx = torch.autocast(device, dtype=torch.bfloat16) if mode == "autocast" else None
        if ctx:
            ctx.__enter__()
        for _ in range(200):
            eval(code, env)
        t = time.perf_counter()
        for _ in range(n):
            eval(code, env)
        if device == "cuda":
            torch.cuda.synchronize()
        out[name] = (time.perf_counter() - t) / n * 1e6
        if ctx:
            ctx.__exit__(None, None, None)
    print(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--child", default=None)
    a = ap.parse_args()
    if a.child:
        return run(a.child, a.device, a.n)
    res = {}
    for mode in ("plain", "amp_o1", "autocast"):
        r = subprocess.run([sys.executable, __file__, "--child", mode, "--device", a.device, "--n", str(a.n)],
                           capture_output=True, text=True, check=True)
        res[mode] = json.loads(r.stdout.strip().splitlines()[-1])
    rows = []
    for name in CASES:
        p, o, ac = res["plain"][name], res["amp_o1"][name], res["autocast"][name]
        rows.append({"op": name, "plain_us": round(p, 2), "amp_o1_us": round(o, 2), "autocast_us": round(ac, 2),
                     "o1_overhead_us": round(o - p, 2), "autocast_overhead_us": round(ac - p, 2)})
    print(json.dumps({"device": a.device, "per_call": rows}, indent=1))


if __name__ == "__main__":
    main()
