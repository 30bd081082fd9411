"""Per-kernel duration / grid-size histogram from a rocprofv3 --output-format csv kernel trace.

  python tools/trace_sizes.py <run_kernel_trace.csv> <name-substring> [...]

For each matching kernel name prints call count, total ms and the (grid size, count, mean us)
groups — which call sites a generic kernel (an elementwise add, a fill) comes from.
"""
import csv
import sys
from collections import defaultdict


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    groups = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if not any(s in name for s in subs):
            continue
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        groups[name[:120]][int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)].append(dur)
    for name, by in groups.items():
        tot = sum(sum(v) for v in by.values())
        print(f"== {name}: {sum(len(v) for v in by.values())} calls, {tot / 1e3:.1f} ms")
        for g, v in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:12]:
            print(f"   grid {g:>10}: {len(v):6d} calls, mean {sum(v) / len(v):9.1f} us, total {sum(v) / 1e3:8.1f} ms")


if __name__ == "__main__":
    main()
