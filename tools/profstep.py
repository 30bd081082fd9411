"""Per-step kernel breakdown from a rocprofv3 kernel trace, restricted to the LAST k steps.

The summary CSV of `rocprofv3 --stats` mixes warmup and setup kernels (synthetic data
generation, first-iteration bucket layout) into its totals. This reads the per-dispatch
`*_kernel_trace.csv` instead and keeps only the dispatches inside the last k training steps,
using the optimizer's final kernel (LAMB stage 2 by default) as the step boundary.

  python tools/profstep.py <kernel_trace.csv> [k=3] [top=30] [boundary=lamb_stage2] [skip=0]
(skip: leave out the last `skip` steps, e.g. to read the bf16 pass of a `bench.py --fp8` trace)
Prints ms/step per kernel name (summed over dispatches), the step wall span and the GPU-busy
fraction (sum of kernel time / span).
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    boundary = sys.argv[4] if len(sys.argv) > 4 else "lamb_stage2"
    skip = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if boundary in r["Kernel_Name"]]
    # a step may launch the boundary kernel more than once (one per param group): group launches
    # closer than 1 ms
    steps = []
    for i in ends:
        if steps and int(rows[i]["Start_Timestamp"]) - int(rows[steps[-1]]["End_Timestamp"]) < 1_000_000:
            steps[-1] = i
        else:
            steps.append(i)
    if skip:
        steps = steps[:-skip]
    if len(steps) < k + 1:
        raise SystemExit(f"only {len(steps)} step boundaries found")
    lo, hi = steps[-k - 1] + 1, steps[-1] + 1
    sel = rows[lo:hi]
    span = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e6 / k
    agg = defaultdict(lambda: [0.0, 0])
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        a = agg[r["Kernel_Name"]]
        a[0] += d
        a[1] += 1
    tot = sum(v[0] for v in agg.values()) / k
    print(f"last {k} steps: span {span:.2f} ms/step, kernel time {tot:.2f} ms/step ({100 * tot / span:.1f}% busy), "
          f"{len(sel) / k:.0f} dispatches/step")
    for name, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{t / k:8.3f} ms/step {100 * t / k / tot:6.2f}% n/step={n / k:6.1f} avg={1e3 * t / n:8.1f}us {name[:100]}")


if __name__ == "__main__":
    main()
