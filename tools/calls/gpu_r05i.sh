#!/bin/bash
# round 5, call 10: wave-split remainder GEMM on a side stream beside the following LayerNorm (tools/overlap_rem_ln.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05i; mkdir -p $O
timeout -k 10 300 python3 -u tools/overlap_rem_ln.py > $O/overlap_rem_ln.txt 2>&1; rc=$?
cat $O/overlap_rem_ln.txt; exit $rc
