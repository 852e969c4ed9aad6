#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel_stats.csv: per-kernel total/avg time, per-step share."""
import csv
import sys


def main(path, steps=None, top=30):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{'total ms':>9} {'%':>6} {'calls':>6} {'avg us':>9}  kernel")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print(f"{float(r['TotalDurationNs'])/1e6:9.2f} {float(r['Percentage']):6.2f} {r['Calls']:>6} "
              f"{float(r['AverageNs'])/1e3:9.1f}  {r['Name'][:140]}")
    print(f"sum of kernel time: {tot/1e6:.2f} ms" + (f" = {tot/1e6/steps:.2f} ms/step over {steps} steps" if steps else ""))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
