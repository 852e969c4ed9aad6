#!/usr/bin/env python3
"""Summarise tools/gemm_diag stamps of the ping-pong GEMM: per-k-tile phase durations per group.

group 0 stamps: start, pre-loop, then per k-tile j: [after mem(j), after end_even, after end_odd], end-loop, end.
group 1 stamps: start, pre-loop, after first end_even, then per j: [after mem(j), after end_odd, after end_even],
                end-loop, end.
"""
import statistics
import sys


def main(path):
    lines = open(path).read().splitlines()
    print(lines[0])
    g = {}
    for ln in lines[1:]:
        if ln.startswith("group"):
            k = int(ln.split()[1])
            g[k] = [int(x) for x in ln.split(":")[1].split()]
    s0 = g[0]
    body = s0[2:-2]
    nk = len(body) // 3
    mem, wait_even, comp = [], [], []
    prev = s0[1]
    for j in range(nk):
        a, b, c = body[3 * j:3 * j + 3]
        mem.append(a - prev)       # issue + ds_reads + lgkmcnt
        wait_even.append(b - a)    # barrier wait after mem (partner computing)
        comp.append(c - b)         # MFMA issue + end_odd wait + barrier
        prev = c
    print(f"group0: prologue {s0[1] - s0[0]} cyc, k-loop {s0[-2] - s0[1]} cyc for {nk} k-tiles "
          f"({(s0[-2] - s0[1]) / max(nk, 1):.0f}/k-tile), epilogue {s0[-1] - s0[-2]} cyc")
    for name, v in (("mem(issue+reads)", mem), ("barrier wait after mem", wait_even), ("compute+end_odd", comp)):
        print(f"  {name:24s} median {statistics.median(v):7.0f}  mean {statistics.mean(v):7.0f}  "
              f"min {min(v):6d}  max {max(v):6d}")
    if 1 in g:
        s1 = g[1]
        body = s1[3:-2]
        nk1 = len(body) // 3
        mem1, wodd, comp1 = [], [], []
        prev = s1[2]
        for j in range(nk1):
            a, b, c = body[3 * j:3 * j + 3]
            mem1.append(a - prev)
            wodd.append(b - a)
            comp1.append(c - b)
            prev = c
        print(f"group1: k-loop {s1[-2] - s1[1]} cyc")
        for name, v in (("mem(reads)", mem1), ("end_odd wait", wodd), ("issue+compute+barrier", comp1)):
            if v:
                print(f"  {name:24s} median {statistics.median(v):7.0f}  mean {statistics.mean(v):7.0f}  "
                      f"min {min(v):6d}  max {max(v):6d}")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
