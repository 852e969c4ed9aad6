#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -x -q --timeout 150 --timeout-method thread -k "attention or c1 or trajectory" > gpurun_out/t_dbg2.log 2>&1
echo "rc=$? $(tail -1 gpurun_out/t_dbg2.log)"
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_ab.log 2>&1 || { tail -5 gpurun_out/b_ab.log; exit 1; }
echo "$(tail -1 gpurun_out/b_ab.log | grep -o '"value": [0-9.]*')"
done
bash tools/ktrace.sh > /dev/null 2>&1; grep attn gpurun_out/kt/step_timeline.txt
