"""Summarise the rocprofv3 counter passes of tools/gpu_gemm_pmc.sh: the GEMM dispatches of
`tools/gemm_energy_vs_lib.py run 3` come in a fixed order (SHAPES x [hipblaslt, apex_persist] x 3
reps), so each group of 3 consecutive GEMM dispatches is labelled by position; per (shape, impl) the
median of each counter, plus per-MFMA ratios.  python tools/pmc_gemm_summary.py <dir>"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_energy_vs_lib import SHAPES  # noqa: E402

IMPLS = ["hipblaslt", "apex_persist"]
REPS = 3


def main(d):
    out = collections.defaultdict(dict)
    names = {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        rows = list(csv.DictReader(open(f)))
        disp = collections.OrderedDict()
        for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
            n = r["Kernel_Name"]
            if "gemm_persist" not in n and "Cijk" not in n:
                continue
            disp.setdefault(int(r["Dispatch_Id"]), (n, {}))[1][r["Counter_Name"]] = \
                disp.get(int(r["Dispatch_Id"]), (n, {}))[1].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        ids = list(disp)
        labels = [(s[0], impl) for s in SHAPES for impl in IMPLS]
        if len(ids) != len(labels) * REPS:
            print(f"warning: {f}: {len(ids)} GEMM dispatches, expected {len(labels) * REPS}", file=sys.stderr)
            continue
        for gi, lab in enumerate(labels):
            grp = [disp[i] for i in ids[gi * REPS:(gi + 1) * REPS]]
            names["%s|%s" % lab] = grp[0][0][:90]
            for c in grp[0][1]:
                v = sorted(g[1][c] for g in grp)
                out["%s|%s" % lab][c] = v[len(v) // 2]
    for k, v in out.items():
        v["kernel"] = names.get(k)
        m = v.get("SQ_INSTS_MFMA")
        if m:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_LDS_IDX_ACTIVE",
                      "SQ_LDS_BANK_CONFLICT"):
                if c in v:
                    v[c + "_per_mfma"] = round(v[c] / m, 4)
        if "TCC_HIT_sum" in v and "TCC_MISS_sum" in v:
            v["l2_hit_rate"] = round(v["TCC_HIT_sum"] / max(1.0, v["TCC_HIT_sum"] + v["TCC_MISS_sum"]), 4)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
