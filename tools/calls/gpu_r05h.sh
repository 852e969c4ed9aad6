#!/bin/bash
# round 5, call 9: the per-rank shapes of the DP configs and Res-ViT on the round's GEMM changes (in-place weights,
# split-K weight gradients on the half-tile kernel), against 870f926 (abase) on the same box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
for a in "l16 --batch 64" "h14 --batch 128" "resvit_b16"; do
  t=$(echo $a | cut -d' ' -f1)
  (cd abase && timeout -k 10 400 python3 -u bench.py --arch $a --steps 10 --warmup 3 --no-cpu-baseline > ../$O/base_$t.json 2> ../$O/base_$t.err) || { tail -3 $O/base_$t.err; exit 1; }
  timeout -k 10 400 python3 -u bench.py --arch $a --steps 10 --warmup 3 --no-cpu-baseline > $O/new_$t.json 2> $O/new_$t.err || { tail -3 $O/new_$t.err; exit 1; }
  echo "$t base: $(grep -o '"value": [0-9.]*' $O/base_$t.json | head -1)  new: $(grep -o '"value": [0-9.]*' $O/new_$t.json | head -1)"
done
