#!/bin/bash
# round 5, call 11: kernel-trace timeline of the overlapped remainder / LayerNorm pairs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05j; mkdir -p $O
OVERLAP_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 -u tools/overlap_rem_ln.py > $O/log.txt 2>&1 || { tail -20 $O/log.txt; exit 1; }
f=$(ls $O/trace/*/*kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find $O/trace -name '*kernel_trace.csv' | head -1)
python3 - "$f" <<'P'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
keep = [r for r in rows if any(k in r["Kernel_Name"] for k in ("gemm", "ln_"))][-40:]
t0 = int(keep[0]["Start_Timestamp"])
for r in keep:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f'{s/1e3:9.1f} {e/1e3:9.1f} {(e-s)/1e3:7.1f} q{r.get("Queue_Id","?")} s{r.get("Stream_Id","?")} {r["Kernel_Name"][:70]}')
P
