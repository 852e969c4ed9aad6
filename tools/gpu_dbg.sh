#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_resvit_gpu.py tests/test_resvit_train_gpu.py -v --timeout 250 --timeout-method thread > gpurun_out/t_dbg.log 2>&1
rc=$?; grep -E "FAIL|passed|failed" gpurun_out/t_dbg.log | tail -5
timeout -k 10 300 python -u bench.py --arch resvit_b16 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b_resvit.log 2>&1 || { tail -5 gpurun_out/b_resvit.log; exit 1; }
tail -1 gpurun_out/b_resvit.log | cut -c1-200
O=gpurun_out/kt_resvit; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- python3 bench.py --arch resvit_b16 --steps 3 --warmup 2 --no-cpu-baseline > $O/ktrace.log 2>&1 || { echo FAILED; tail -5 $O/ktrace.log; exit 1; }
S=$(find $O/ktrace -name "*kernel_stats.csv" | head -1)
T=$(find $O/ktrace -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py $S 5 > $O/kernel_summary.txt
python3 tools/trace_step.py $T 1 $O/step_launches.txt > $O/step_timeline.txt
rm -rf $O/ktrace
head -3 $O/step_timeline.txt
exit $rc
