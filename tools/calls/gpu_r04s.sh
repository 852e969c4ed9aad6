#!/bin/bash
# round 4, call 20: launch-gap probe (tools/gap_probe.py) under a kernel trace: idle time in front of each kernel
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/gap_probe.py > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
T=$(find $O/kt -name "*kernel_trace.csv" | head -1)
cp $T $O/kernel_trace.csv
python3 - $O/kernel_trace.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
prev = None
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "")[:48]
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (st - prev) / 1000 if prev else 0
    print(f"{gap:9.2f} us gap  {(en - st) / 1000:8.1f} us  {name}")
    prev = en
PY
