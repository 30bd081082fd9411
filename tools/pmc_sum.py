"""Summarise one rocprofv3 --pmc counter_collection.csv: per kernel (full demangled name, so
template variants stay apart) the median per-dispatch counters plus LDS instructions per MFMA
instruction and the bank-conflict share of LDS cycles.

    python tools/pmc_sum.py path/to/p_counter_collection.csv
"""
import csv
import json
import statistics
import sys
from collections import defaultdict


def main():
    data = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(sys.argv[1])):
        name = r["Kernel_Name"]
        if "fill_kernel" in name:
            continue
        data[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in data.items():
        m = {c: statistics.median(v) for c, v in cs.items()}
        if m.get("SQ_INSTS_MFMA"):
            m["lds_per_mfma"] = round(m.get("SQ_INSTS_LDS", 0) / m["SQ_INSTS_MFMA"], 3)
        if m.get("SQ_LDS_IDX_ACTIVE"):
            m["lds_conflict_pct"] = round(100.0 * m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"], 2)
        out[k] = m
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
