#!/bin/bash
# round 6, call 2: the 4-wave 128x128-per-wave prototype (tools/w4_proto.hip) on the B/16 N = 768 / 3072 shapes,
# beside the library's kernels on the same box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b; mkdir -p $O
step() { echo "== $1"; shift; "$@" || { echo "FAILED: $*"; exit 1; }; }
for sh in "50432 768 2304" "50432 768 3072" "50432 768 768" "50432 3072 768"; do
  step "proto $sh" timeout -k 10 120 tools/w4_proto $sh >> $O/proto.txt 2>&1
done
cat $O/proto.txt
step "gemm_bench" timeout -k 10 300 python3 -u tools/gemm_bench.py --tiles 0 --blas --rounds 3 \
  --shapes qkvdg:1,fc1dgk:1,outk:1,fc2dgk:1 > $O/gemm_bench.txt 2>&1
cat $O/gemm_bench.txt
