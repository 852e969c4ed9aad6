#!/bin/bash
# round 5, call 33: evidence set v2 on the current tree: full -m gpu suite, smoke, B/16 bench + kernel trace + PMC
# passes (tools/prof_r05.sh v2), then the Res-ViT-B/16 bench line
set -o pipefail
export TMPDIR=/tmp
bash tools/prof_r05.sh v2 || exit 1
O=gpurun_out/r05_prof_v2
timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 20 --warmup 5 > $O/bench_resvit_b16.json 2> $O/bench_resvit_b16.err || { tail -5 $O/bench_resvit_b16.err; exit 1; }
tail -c 300 $O/bench_resvit_b16.json
