#!/bin/bash
# bench A/B of VIT_GEMM_PRIO (s_setprio around the ping-pong MFMA clusters), alternately on one box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prio; mkdir -p $O
for i in 1 2; do
  for e in 0 1; do
    VIT_GEMM_PRIO=$e timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b${e}_$i.json 2> $O/b${e}_$i.err || { tail -3 $O/b${e}_$i.err; exit 1; }
    echo "prio=$e: $(grep -o '"value": [0-9.]*' $O/b${e}_$i.json) $(grep -o '"frac": [0-9.]*' $O/b${e}_$i.json | head -1)"
  done
done
