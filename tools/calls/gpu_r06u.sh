#!/bin/bash
# round 6, call 21: split-K weight gradient with one K-contiguous operand vs both M/N-contiguous (what a feature-major
# copy of one activation would buy)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 300 python3 -u tools/dbg/wgrad_layout_bench.py > $O/wgrad_layout.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/wgrad_layout.txt
exit $rc
