"""Summarise tools/gpu_pmc_bw.sh: per kernel, the median FETCH_SIZE / WRITE_SIZE per dispatch
(rocprofv3 reports both in KB) and the median dispatch time of the counter runs, giving the
counter-measured bytes and HBM-side GB/s next to the op timings of tools/bw_kernels.py.

    python tools/pmc_bw_summary.py gpurun_out/pmc_bw > summary.json
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def _short(name):
    n = name.split("(")[0]
    for pre in ("void ", "apex::", "(anonymous namespace)::"):
        n = n.replace(pre, "")
    return n[:80]


def main():
    d = sys.argv[1]
    per = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = _short(r["Kernel_Name"])
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if "Start_Timestamp" in r and r["Start_Timestamp"]:
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    timing = []
    tf = os.path.join(d, "timing.jsonl")
    if os.path.exists(tf):
        timing = [json.loads(l) for l in open(tf) if l.startswith("{")]
    out = {"note": "median per dispatch; FETCH/WRITE in MB (rocprofv3 KB / 1024); us from the counter runs' "
                   "dispatch timestamps; GBps = (fetch + write) / us", "ops": timing, "kernels": {}}
    for k, cs in sorted(per.items()):
        if "FETCH_SIZE" not in cs and "WRITE_SIZE" not in cs:
            continue
        e = {c: round(statistics.median(v) / 1024.0, 3) for c, v in cs.items() if c in ("FETCH_SIZE", "WRITE_SIZE")}
        if "GRBM_GUI_ACTIVE" in cs:
            e["GRBM_GUI_ACTIVE"] = statistics.median(cs["GRBM_GUI_ACTIVE"])
        e["dispatches"] = max(len(v) for v in cs.values())
        if dur[k]:
            us = statistics.median(dur[k])
            e["us"] = round(us, 1)
            e["GBps"] = round((e.get("FETCH_SIZE", 0) + e.get("WRITE_SIZE", 0)) * 1.048576e6 / us / 1e3, 1) if us else None
        out["kernels"][k] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
