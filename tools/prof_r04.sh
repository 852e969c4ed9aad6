#!/bin/bash
# Round-4 evidence for profiles/r04/: bench lines with rocprofv3 kernel traces and step timelines for the
# shapes the DP configs run per rank (C3: ViT-L/16 bs 64, C4: ViT-H/14 bs 128) and for Res-ViT-B/16 (C5).
# usage: bash tools/prof_r04.sh TAG "l16:64 h14:128 resvit_b16:128"
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-v1}
O=gpurun_out/r04_$TAG
mkdir -p $O
for spec in ${2:-l16:64 h14:128 resvit_b16:128}; do
  arch=${spec%%:*}; bs=${spec##*:}
  n=${arch}_bs${bs}
  echo "== $n"
  timeout -k 10 300 python3 -u bench.py --arch $arch --batch $bs --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err || { tail -5 $O/bench_$n.err; exit 1; }
  tail -c 300 $O/bench_$n.json; echo
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$n -o run -- python3 bench.py --arch $arch --batch $bs --steps 6 --warmup 2 --no-cpu-baseline > $O/kt_$n.log 2>&1 || { tail -5 $O/kt_$n.log; exit 1; }
  S=$(find $O/kt_$n -name "*kernel_stats.csv" | head -1)
  T=$(find $O/kt_$n -name "*kernel_trace.csv" | head -1)
  python3 tools/prof_summary.py $S 8 > $O/summary_$n.txt
  python3 tools/trace_step.py $T 2 $O/launches_$n.txt > $O/timeline_$n.txt
  rm -rf $O/kt_$n
  head -16 $O/timeline_$n.txt
done
