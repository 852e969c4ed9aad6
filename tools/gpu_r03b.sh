#!/bin/bash
# round 3 re-entry: full GPU suite, default bench line (with CPU baseline), Res-ViT bench line,
# kernel trace of the default step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; tail -3 $O/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_b16.json 2> $O/bench_b16.err || { tail -5 $O/bench_b16.err; exit 1; }
tail -c 300 $O/bench_b16.json; echo
timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_resvit.json 2> $O/bench_resvit.err || { tail -5 $O/bench_resvit.err; exit 1; }
tail -c 300 $O/bench_resvit.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/ktrace.log 2>&1 || { echo KTRACE FAILED; tail -5 $O/ktrace.log; exit 1; }
S=$(find $O/ktrace -name "*kernel_stats.csv" | head -1)
T=$(find $O/ktrace -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py $S 13 > $O/kernel_summary.txt
python3 tools/trace_step.py $T 1 $O/step_launches.txt > $O/step_timeline.txt
rm -rf $O/ktrace
head -40 $O/step_timeline.txt
