#!/bin/bash
# attention + parity GPU tests, then the default bench line twice
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_new_$i.log 2>&1 || exit 1
tail -1 gpurun_out/b_new_$i.log | grep -o '"value": [0-9.]*'
done
