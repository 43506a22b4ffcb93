"""Per-plan-kernel table of arbitrary rocprofv3 PMC counters (one or more
*_counter_collection.csv files from `rocprofv3 --pmc ...` runs of bench.py).

  python tools/pmc_table.py DIR1/x_counter_collection.csv [DIR2/y_counter_collection.csv ...] [--out F.json]

Dispatches are attributed to plan kernels by position inside each forward, as in
prof_summary.py.  Derived columns (when their inputs were collected):
  clk_ghz   GRBM_GUI_ACTIVE / 8 XCDs / kernel duration — the effective shader clock
  mfma_util SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 4 SIMD * 256 CU)
"""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import prof_summary as P  # noqa: E402


def table(paths):
    res = defaultdict(dict)
    for path in paths:
        rows = list(csv.DictReader(open(path)))
        by_counter = defaultdict(list)
        for r in rows:
            by_counter[r["Counter_Name"]].append(r)
        for cname, crows in by_counter.items():
            vals = defaultdict(list)
            for pk, r in P.dispatch_sequence(crows):
                vals[pk].append(float(r["Counter_Value"]))
            for pk, v in vals.items():
                res[pk][cname] = sum(v) / len(v)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--trace", help="kernel trace csv for durations (clk_ghz)")
    ap.add_argument("--out")
    ap.add_argument("--fp16", action="store_true", help="fp16 plan kernel order")
    a = ap.parse_args()
    if a.fp16:
        P.ORDER[:] = P.ORDER_FP16
    res = table(a.csv)
    if a.trace:
        s = P.summarise(a.trace)
        for pk, d in s.items():
            res[pk]["avg_us"] = d.get("avg_us")
    for pk, d in res.items():
        if "GRBM_GUI_ACTIVE" in d and d.get("avg_us"):
            d["clk_ghz"] = round(d["GRBM_GUI_ACTIVE"] / 8 / (d["avg_us"] * 1e3), 3)
        if "GRBM_GUI_ACTIVE" in d and "SQ_VALU_MFMA_BUSY_CYCLES" in d:
            d["mfma_util"] = round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / (d["GRBM_GUI_ACTIVE"] / 8 * 4 * 256), 4)
    out = {pk: res[pk] for pk in P.ORDER if pk in res}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    cols = sorted({c for d in out.values() for c in d})
    print("kernel        " + " ".join(f"{c[:22]:>22s}" for c in cols))
    for pk, d in out.items():
        print(f"{pk:14s}" + " ".join(f"{d.get(c, float('nan')):22.4g}" for c in cols))


if __name__ == "__main__":
    main()
