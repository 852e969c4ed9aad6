#!/usr/bin/env python3
"""Average each counter over the dispatches of counter_collection.csv files (skip the warm-up ones),
plus the dispatch duration and derived clock / MFMA utilisation (gfx950: 256 CUs x 4 SIMDs).

usage: pmc_table.py FILE.csv [FILE.csv ...] [--kernel SUBSTRING]
"""
import csv
import sys
from collections import defaultdict


def main(argv):
    kern = None
    if "--kernel" in argv:
        i = argv.index("--kernel")
        kern = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    agg = {}
    dur = []
    for path in argv:
        per = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(path)):
            if kern and kern not in r["Kernel_Name"]:
                continue
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                dur.append((int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9))
        for c, d in per.items():
            vals = [d[k] for k in sorted(d, key=int)][3:] or list(d.values())
            agg[c] = sum(vals) / len(vals)
            print(f"{c:28s} {agg[c]:16.1f}")
    if dur:
        dur = [t for _, t in sorted(dur)][3:] or [t for _, t in dur]
        w = sum(dur) / len(dur)
        clk = agg["GRBM_GUI_ACTIVE"] / 8 / w
        print(f"{'duration_us':28s} {w * 1e6:16.1f}")
        print(f"{'clock_GHz':28s} {clk / 1e9:16.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in agg:
            print(f"{'mfma_util':28s} {agg['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * agg['GRBM_GUI_ACTIVE'] / 8):16.3f}")


if __name__ == "__main__":
    main(sys.argv[1:])
