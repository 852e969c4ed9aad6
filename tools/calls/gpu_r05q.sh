#!/bin/bash
# round 5, call 18: Res-ViT-B/16 bs 128 kernel trace after the router / approximator batching
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --arch resvit_b16 --steps 6 --warmup 3 --no-cpu-baseline > $O/ktrace.log 2>&1 || { tail -20 $O/ktrace.log; exit 1; }
S=$(find $O/kt -name "*kernel_stats.csv" | head -1)
T=$(find $O/kt -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py $S 40 > $O/kernel_summary.txt
python3 tools/trace_step.py $T 4 $O/step_launches.txt > $O/step_timeline.txt
rm -rf $O/kt
grep -o '"value": [0-9.]*' $O/ktrace.log | head -1
head -45 $O/kernel_summary.txt; head -5 $O/step_timeline.txt
