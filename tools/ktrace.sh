#!/bin/bash
# kernel trace of the default bench step -> gpurun_out/kt/{kernel_summary,step_timeline}.txt
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/kt
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > $O/ktrace.log 2>&1 || { echo FAILED; tail -5 $O/ktrace.log; exit 1; }
S=$(find $O/ktrace -name "*kernel_stats.csv" | head -1)
T=$(find $O/ktrace -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py $S 13 > $O/kernel_summary.txt
python3 tools/trace_step.py $T 1 $O/step_launches.txt > $O/step_timeline.txt
cp $S $O/kernel_stats.csv
rm -rf $O/ktrace
tail -1 $O/ktrace.log | cut -c1-120
