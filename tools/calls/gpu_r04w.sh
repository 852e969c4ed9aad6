#!/bin/bash
# round 4, call 23: Res-ViT router backward: the global half of out_conv's input gradient through its token sum (linearity):
# Res-ViT GPU tests (router parity vs the fp32 per-op router and the reference), then Res-ViT-B/16 bs 128 bench
# against the round-4 bench line on another box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_resvit_train_gpu.py tests/test_resvit_gpu.py -x -q -rP --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 20 --warmup 3 --no-cpu-baseline > $O/new_$r.json 2> $O/new_$r.err || { tail -3 $O/new_$r.err; exit 1; }
  echo "router global-half by token sum $r: $(grep -o '"value": [0-9.]*' $O/new_$r.json | head -1)"
done
