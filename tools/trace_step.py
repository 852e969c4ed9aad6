#!/usr/bin/env python3
"""Per-step timeline view of a rocprofv3 kernel_trace.csv of bench.py.

Splits the trace into steps at the SGD kernel, takes the chosen step (bench.py: 2 = the last timed step; 1 is the
probe step after the timed region, whose HIP events around the roofline kernels add ~6 us of idle each), and
reports per stream:
busy time (union of kernel intervals), and per kernel class the summed duration, plus the step's
wall span and the time during which NO kernel runs (launch gaps / host waits).
usage: trace_step.py run_kernel_trace.csv [step_index_from_end=1] [launch_list_out]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"::(\w+)<([^>]*)>", name) or re.search(r"::(\w+)\(", name)
    if not m:
        return name[:60]
    base = m.group(1)
    if base.startswith("gemm_") and m.lastindex and m.lastindex >= 2:
        args = [a.strip() for a in m.group(2).split(",")]
        return f"{base}<...,{','.join(args[-3:])}>"
    return base


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sgd = [i for i, r in enumerate(rows) if ("sgd_kernel" in r["Kernel_Name"] or "sgd_dev_kernel" in r["Kernel_Name"]) or "adamw_update_kernel" in r["Kernel_Name"]]
    lo, hi = sgd[-k - 1] + 1, sgd[-k] + 1
    step = rows[lo:hi]
    t0 = min(int(r["Start_Timestamp"]) for r in step)
    t1 = max(int(r["End_Timestamp"]) for r in step)
    print(f"step wall span: {(t1 - t0) / 1e3:.1f} us, {len(step)} kernels")
    allv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step]
    print(f"GPU busy (any kernel): {union(allv) / 1e3:.1f} us; idle {(t1 - t0 - union(allv)) / 1e3:.1f} us")
    by_q = defaultdict(list)
    for r in step:
        by_q[r["Queue_Id"]].append(r)
    for q, rs in by_q.items():
        iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rs]
        print(f"queue {q}: {len(rs)} kernels, busy {union(iv) / 1e3:.1f} us")
        cls = defaultdict(lambda: [0, 0])
        for r in rs:
            c = cls[short(r["Kernel_Name"])]
            c[0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            c[1] += 1
        for name, (d, n) in sorted(cls.items(), key=lambda x: -x[1][0]):
            print(f"   {d / 1e3:9.1f} us  {n:4d}x  {d / n / 1e3:8.1f} avg  {name}")
    if len(sys.argv) > 3:  # the step's launches in issue order: start offset, duration, queue, kernel
        with open(sys.argv[3], "w") as f:
            for r in step:
                s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                f.write(f"{(s0 - t0) / 1e3:9.1f} {(e0 - s0) / 1e3:8.1f} q{r['Queue_Id']} {short(r['Kernel_Name'])}\n")


if __name__ == "__main__":
    main()
