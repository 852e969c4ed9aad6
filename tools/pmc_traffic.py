#!/usr/bin/env python3
"""Per-launch HBM traffic of one kernel from rocprofv3 --pmc counter_collection.csv files.

Usage: pmc_traffic.py NAME_REGEX fetch.csv write.csv [out.json]
FETCH_SIZE / WRITE_SIZE are in KB. gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports
half the bytes of wide coalesced streaming reads (16 B/lane global_load and buffer_load ... lds), so it is
doubled; WRITE_SIZE is exact for 16 B/lane streaming stores.
"""
import csv
import json
import re
import sys
from collections import defaultdict


def per_dispatch(path, counter, rx):
    vals = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or not rx.search(r["Kernel_Name"]):
            continue
        vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    return vals, names


def main():
    rx = re.compile(sys.argv[1])
    f, fn = per_dispatch(sys.argv[2], "FETCH_SIZE", rx)
    w, _ = per_dispatch(sys.argv[3], "WRITE_SIZE", rx)
    assert f and w, "no matching dispatches"
    fetch_b = 2.0 * 1024 * sum(f.values()) / len(f)
    write_b = 1024 * sum(w.values()) / len(w)
    out = {"kernel": next(iter(fn.values())), "dispatches_fetch": len(f), "dispatches_write": len(w),
           "fetch_bytes_raw": fetch_b / 2, "fetch_bytes_corrected": fetch_b, "write_bytes": write_b,
           "traffic_bytes": fetch_b + write_b,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE as reported; KB=1024 B"}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 4:
        json.dump(out, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
