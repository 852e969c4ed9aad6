#!/usr/bin/env python3
"""Per-kernel PMC table over the rocprofv3 --pmc passes of one workload (counter_collection.csv files,
one pass per counter set): launches, average duration, MFMA busy fraction, HBM fetch / write per launch
and the achieved HBM rate, for the kernels with the most total time.

gfx950 conventions (MI355X_MICROARCH.md): SQ_VALU_MFMA_BUSY_CYCLES summed over the 1024 SIMDs, GRBM_GUI_ACTIVE
summed over the 8 XCDs; FETCH_SIZE / WRITE_SIZE in KB, FETCH_SIZE doubled for the wide-read undercount.

usage: kernel_pmc.py OUT.txt FILE.csv [FILE.csv ...]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = re.sub(r"\(.*$", "", n)
    return n[:70]


def main(out, files):
    cnt = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> dispatch -> value
    dur = defaultdict(dict)
    for path in files:
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            d = r["Dispatch_Id"]
            cnt[k][r["Counter_Name"]][(path, d)] += float(r["Counter_Value"])
            dur[k][(path, d)] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    rows = []
    for k, cs in cnt.items():
        avg = {c: sum(v.values()) / len(v) for c, v in cs.items()}
        ds = list(dur[k].values())
        t = sum(ds) / len(ds)
        n = max(len(v) for v in cs.values())
        rows.append((t * n, k, n, t, avg))
    rows.sort(reverse=True)
    lines = [f"{'kernel':70s} {'launch':>6} {'avg us':>8} {'mfma':>6} {'fetch MB':>9} {'write MB':>9} {'HBM TB/s':>8}"]
    for _, k, n, t, a in rows[:25]:
        cyc = a.get("GRBM_GUI_ACTIVE", 0) / 8
        mf = a["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc) if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in a else float("nan")
        fe = a.get("FETCH_SIZE", float("nan")) * 2 / 1024
        wr = a.get("WRITE_SIZE", float("nan")) / 1024
        bw = (fe + wr) * 1048576 / t / 1e12 if t else float("nan")
        lines.append(f"{k:70s} {n:6d} {t * 1e6:8.1f} {mf:6.3f} {fe:9.1f} {wr:9.1f} {bw:8.2f}")
    txt = "\n".join(lines)
    open(out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
