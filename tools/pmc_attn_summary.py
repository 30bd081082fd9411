"""Summarise tools/gpu_attn_pmc2.sh: per (shape, pass, kernel) the median per-dispatch counters
and derived ratios — MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES over every SIMD's cycles:
GRBM_GUI_ACTIVE is summed over the 8 XCDs, 1024 SIMDs in all), VALU and LDS instructions per
MFMA instruction, and the LDS bank-conflict share of LDS cycles.

    python tools/pmc_attn_summary.py gpurun_out/apmc2 > summary.json
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    data = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "*_p*", "**", "*counter_collection.csv"), recursive=True):
        case = os.path.basename(os.path.dirname(f) if "_p" in os.path.basename(os.path.dirname(f)) else
                                os.path.dirname(os.path.dirname(f)))
        case = case.rsplit("_p", 1)[0]
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "attn" not in name:
                continue
            k = case + " :: " + ("fwd" if "fwd" in name else "bwd_dq" if "dq_kernel" in name else "bwd")
            data[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in sorted(data.items()):
        m = {c: statistics.median(v) for c, v in cs.items()}
        e = dict(m)
        g = m.get("GRBM_GUI_ACTIVE") or m.get("GRBM_COUNT")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            e["mfma_busy_pct"] = round(100.0 * m["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 1024), 1)
        if m.get("SQ_INSTS_MFMA"):
            e["valu_per_mfma"] = round(m.get("SQ_INSTS_VALU", 0) / m["SQ_INSTS_MFMA"], 2)
            e["lds_per_mfma"] = round(m.get("SQ_INSTS_LDS", 0) / m["SQ_INSTS_MFMA"], 2)
        if m.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_conflict_pct"] = round(100.0 * m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"], 1)
        out[k] = e
    print(json.dumps({"note": "median per dispatch over 4-5 launches; see tools/pmc_attn_summary.py", "kernels": out},
                     indent=1))


if __name__ == "__main__":
    main()
