#!/bin/bash
# A/B: bias-gradient partial buffer ring depth
set -o pipefail
export TMPDIR=/tmp
for i in 1 2; do
for nb in 2 4 8; do
VITMI_BIAS_BUFS=$nb timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_ab.log 2>&1 || { tail -5 gpurun_out/b_ab.log; exit 1; }
echo "bufs=$nb $(tail -1 gpurun_out/b_ab.log | grep -o '"value": [0-9.]*')"
done
done
