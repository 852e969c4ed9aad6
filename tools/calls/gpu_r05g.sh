#!/bin/bash
# round 5, call 8: the 128x128 remainder kernel reads M/N-contiguous fragments by inline asm too (the fc1 data
# gradient's remainder with W1 read in place took 60 us): GEMM tests, then a same-box A/B against 870f926
# (before in-place weights and the split-K weight gradients on the half-tile kernel)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py -k "gemm or b16 or step or large" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  (cd abase && timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > ../$O/base_$r.json 2> ../$O/base_$r.err) || { tail -3 $O/base_$r.err; exit 1; }
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/new_$r.json 2> $O/new_$r.err || { tail -3 $O/new_$r.err; exit 1; }
  echo "base $r: $(grep -o '"value": [0-9.]*' $O/base_$r.json | head -1)  new $r: $(grep -o '"value": [0-9.]*' $O/new_$r.json | head -1)"
done
