#!/bin/bash
# round 4, call 28: router-MLP and approximator weight gradients accumulated in place into the flat .grad views
# (vitmi.flat.grad_sink, no AccumulateGrad adds): Res-ViT GPU tests, then Res-ViT-B/16 bs 128 bench
# sinks vs autograd accumulation (VITMI_RESVIT_NO_SINK=1), same box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04sink; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_resvit_train_gpu.py tests/test_resvit_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 20 --warmup 3 --no-cpu-baseline > $O/shared_$r.json 2> $O/shared_$r.err || { tail -3 $O/shared_$r.err; exit 1; }
  VITMI_RESVIT_NO_SINK=1 timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 20 --warmup 3 --no-cpu-baseline > $O/each_$r.json 2> $O/each_$r.err || { tail -3 $O/each_$r.err; exit 1; }
  echo "sink $r: $(grep -o '"value": [0-9.]*' $O/shared_$r.json | head -1)  accum $r: $(grep -o '"value": [0-9.]*' $O/each_$r.json | head -1)"
done
