#!/bin/bash
# round 6, call 5: w4 prototype with A prefetched two k-tiles ahead (w4p) vs one ahead (w4) and LDS-DMA (w4d)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e; mkdir -p $O
step() { echo "== $1"; shift; "$@" || { echo "FAILED: $*"; exit 1; }; }
for sh in "50432 768 3072" "50432 768 2304" "50432 768 768" "50432 3072 768"; do
  step "proto $sh" timeout -k 10 120 tools/w4_proto $sh >> $O/proto.txt 2>&1
done
grep -v "rel fro err 1.6" $O/proto.txt
