#!/bin/bash
# split-K weight-gradient tile config A/B (VIT_GEMM_SPLITK_CFG 5 = 256x256x64 2 buffers, 7 = x32 4 buffers,
# 8 = x32 5 buffers), then VIT_GEMM_PRIO; alternately on one box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/skcfg; mkdir -p $O
VIT_GEMM_SPLITK_CFG=7 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "wgrad or splitk" -x -q --timeout 200 --timeout-method thread > $O/t7.log 2>&1; rc=$?; tail -1 $O/t7.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for c in 5 7 8; do
    VIT_GEMM_SPLITK_CFG=$c timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b${c}_$i.json 2> $O/b${c}_$i.err || { tail -3 $O/b${c}_$i.err; exit 1; }
    echo "cfg=$c: $(grep -o '"value": [0-9.]*' $O/b${c}_$i.json) $(grep -o '"frac": [0-9.]*' $O/b${c}_$i.json | head -1)"
  done
  VIT_GEMM_PRIO=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bp_$i.json 2> $O/bp_$i.err || { tail -3 $O/bp_$i.err; exit 1; }
  echo "cfg=5 prio=1: $(grep -o '"value": [0-9.]*' $O/bp_$i.json) $(grep -o '"frac": [0-9.]*' $O/bp_$i.json | head -1)"
done
