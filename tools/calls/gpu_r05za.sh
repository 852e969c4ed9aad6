#!/bin/bash
# round 5, call 28 (and 31): kernel trace of the current Res-ViT-B/16 bs 128 step (what is left of the ATen glue)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05za; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- python3 bench.py --arch resvit_b16 --steps 6 --warmup 3 --no-cpu-baseline > $O/ktrace.log 2>&1 || { tail -20 $O/ktrace.log; exit 1; }
S=$(find $O/ktrace -name "*kernel_stats.csv" | head -1)
T=$(find $O/ktrace -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py $S 13 > $O/kernel_summary.txt
python3 tools/trace_step.py $T 3 $O/step_launches.txt > $O/step_timeline.txt
rm -rf $O/ktrace
head -3 $O/step_timeline.txt
