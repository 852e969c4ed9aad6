#!/bin/bash
# round 6, call 26: weight-gradient orientation (dW vs dW^T with the operands swapped), production library
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06z; mkdir -p $O
timeout -k 10 300 python3 -u tools/dbg/wgrad_orient_bench.py > $O/orient.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/orient.txt
exit $rc
