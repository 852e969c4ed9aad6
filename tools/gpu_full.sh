#!/bin/bash
# full GPU test suite, then the default bench line twice
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?; tail -2 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_new_$i.log 2>&1 || exit 1
tail -1 gpurun_out/b_new_$i.log | grep -o '"value": [0-9.]*'
done
