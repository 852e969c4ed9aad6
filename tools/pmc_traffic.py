#!/usr/bin/env python3
"""Per-launch HBM traffic of one GEMM call from rocprofv3 --pmc counter_collection.csv files.

A call may launch more than one kernel (the wave split runs the whole-wave rows on a 256x256 kernel
and the remainder on 128x128 tiles): every kernel matching NAME_REGEX is averaged over its own
dispatches and the per-call traffic is the sum over the matched kernels.

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
    w, wn = per_dispatch(sys.argv[3], "WRITE_SIZE", rx)
    assert f and w, "no matching dispatches"
    parts = {}
    for name in sorted(set(fn.values())):
        fd = [v for k, v in f.items() if fn[k] == name]
        wd = [v for k, v in w.items() if wn[k] == name]
        fb = 2.0 * 1024 * sum(fd) / len(fd)
        wb = 1024 * sum(wd) / max(1, len(wd))
        parts[name] = {"dispatches": len(fd), "fetch_bytes_corrected": fb, "write_bytes": wb}
    fetch_b = sum(p["fetch_bytes_corrected"] for p in parts.values())
    write_b = sum(p["write_bytes"] for p in parts.values())
    out = {"kernel": " + ".join(parts), "dispatches_fetch": len(f), "dispatches_write": len(w),
           "fetch_bytes_raw": fetch_b / 2, "fetch_bytes_corrected": fetch_b, "write_bytes": write_b,
           "traffic_bytes": fetch_b + write_b, "per_kernel": parts,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE as reported; KB=1024 B"}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 4:
        json.dump(out, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
