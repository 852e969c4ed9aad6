#!/bin/bash
# round 5, call 39: end-of-round lines of the DP configs' per-rank shapes on one GPU (L/16 bs 64, H/14 bs 128)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zk; mkdir -p $O
timeout -k 10 300 python3 -u bench.py --arch l16 --batch 64 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_l16_bs64.json 2> $O/l16.err || { tail -5 $O/l16.err; exit 1; }
tail -c 250 $O/bench_l16_bs64.json; echo
timeout -k 10 400 python3 -u bench.py --arch h14 --batch 128 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_h14_bs128.json 2> $O/h14.err || { tail -5 $O/h14.err; exit 1; }
tail -c 250 $O/bench_h14_bs128.json; echo
