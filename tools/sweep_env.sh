#!/bin/bash
# A/B of the runtime knobs on the default bench (one gpurun call). Each run has its own time limit;
# the first failure ends the call.   usage: bash tools/sweep_env.sh "VAR=a VAR2=b" "VAR=c" ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
: > $O/sweep.txt
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/sweep_run.log 2>&1 \
    || { tail -20 $O/sweep_run.log; exit 1; }
  v=$(tail -1 $O/sweep_run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')
  echo "[$cfg] img/s ms/step fc1_ms: $v" | tee -a $O/sweep.txt
done
