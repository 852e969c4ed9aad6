#!/bin/bash
# round 6, call 20: the other configurations' bench lines on the final tree (L/16 bs 64, H/14 bs 128: the DP configs'
# per-rank shapes; Res-ViT-B/16 bs 128)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06t; mkdir -p $O
export VITMI_BENCH_TRAIN_EPOCH=0
step() { echo "== $1"; shift; "$@" || { echo "FAILED: $*"; exit 1; }; }
for cfg in "l16 64" "h14 128"; do
  set -- $cfg
  step "bench $1" timeout -k 10 400 python3 -u bench.py --arch $1 --batch $2 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$1_bs$2.json 2> $O/bench_$1.err
  tail -1 $O/bench_$1_bs$2.json | grep -o '"value": [0-9.]*'
done
step "bench resvit" timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_resvit_b16.json 2> $O/bench_resvit.err
tail -1 $O/bench_resvit_b16.json | grep -o '"value": [0-9.]*'
