#!/bin/bash
# A/B of runtime switches on the default bench line: bash tools/bench_env.sh "VAR=a" "VAR=b" ...
export TMPDIR=/tmp
for round in 1 2; do
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_env.log 2>&1 || { echo "FAILED $cfg"; tail -3 gpurun_out/b_env.log; exit 1; }
  echo "$cfg: $(tail -1 gpurun_out/b_env.log | grep -o '"value": [0-9.]*')"
done
done
