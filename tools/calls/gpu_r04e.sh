#!/bin/bash
# round 4, call 5: attention backward stage-2 units two per iteration: tests + standalone A/B against the
# HEAD kernel (vitmi/ab), B/16 bs 256 (full and the pruned layer's q_rows = 1) and L/16 bs 64
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  echo "base:"; VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/ab/libvit_hip.so timeout -k 10 120 python -u tools/attn_bench.py 256 197 12 64 0 64 197 16 64 0 2>&1 | grep bwd
  echo "new:"; timeout -k 10 120 python -u tools/attn_bench.py 256 197 12 64 0 64 197 16 64 0 2>&1 | grep bwd
done
