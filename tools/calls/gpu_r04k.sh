#!/bin/bash
# round 4, call 11: fused Res-ViT approximator step: Res-ViT GPU tests (incl. the bit-exact fused-vs-per-op test),
# then Res-ViT-B/16 bs 128 bench with the fused step and with the per-op approximators (VITMI_RESVIT_APPROX_OPS=1)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_resvit_train_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 20 --warmup 3 --no-cpu-baseline > $O/fused_$r.json 2> $O/fused_$r.err || { tail -3 $O/fused_$r.err; exit 1; }
  VITMI_RESVIT_APPROX_OPS=1 timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 20 --warmup 3 --no-cpu-baseline > $O/ops_$r.json 2> $O/ops_$r.err || { tail -3 $O/ops_$r.err; exit 1; }
  echo "fused $r: $(grep -o '"value": [0-9.]*' $O/fused_$r.json | head -1)  per-op $r: $(grep -o '"value": [0-9.]*' $O/ops_$r.json | head -1)"
done
