#!/bin/bash
# round 6, call 1: hipBLASLt's geometry on the B/16 bs-256 GEMM shapes (kernel names + durations under rocprofv3),
# beside this repo's kernels in the same process
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06a; mkdir -p $O
step() { echo "== $1"; shift; "$@" || { echo "FAILED: $*"; exit 1; }; }
step "gemm_bench" timeout -k 10 300 python3 -u tools/gemm_bench.py --tiles 0 --blas --rounds 3 \
  --shapes fc1:8,fc2:4,outk:1,qkvk:2,fc2dgk:9,fc1dgk:1,qkvdg:1,out:1,qkv:2,fc2dg:9,fc1dg:1 > $O/gemm_bench.txt 2>&1
cat $O/gemm_bench.txt
step "rocprof blas" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o blas -- python3 -u tools/gemm_bench.py --tiles 0 --blas --rounds 1 \
  --shapes fc1:8,fc2:4,outk:1,qkvk:2,fc2dgk:9,fc1dgk:1,qkvdg:1,out:1,qkv:2,fc2dg:9,fc1dg:1 > $O/prof.log 2>&1
find $O/prof -name '*stats*' | head
