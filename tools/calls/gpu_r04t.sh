#!/bin/bash
# round 4, call 21: step timelines of the last TIMED step (trace_step.py step 2; step 1 is bench.py's probe step
# with HIP events around the roofline kernels) for B/16 bs 256, L/16 bs 64, H/14 bs 128, Res-ViT-B/16 bs 128
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04t; rm -rf $O; mkdir -p $O
for spec in ${SPECS:-b16:256 l16:64 h14:128 resvit_b16:128}; do
  arch=${spec%%:*}; bs=${spec##*:}; n=${arch}_bs${bs}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$n -o run -- python3 bench.py --arch $arch --batch $bs --steps 6 --warmup 2 --no-cpu-baseline > $O/kt_$n.log 2>&1 || { tail -5 $O/kt_$n.log; exit 1; }
  T=$(find $O/kt_$n -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_step.py $T 2 $O/launches_$n.txt > $O/timeline_$n.txt
  python3 tools/trace_step.py $T 1 $O/launches_probe_$n.txt > $O/timeline_probe_$n.txt
  rm -rf $O/kt_$n
  echo "== $n"; head -4 $O/timeline_$n.txt; echo "(probe step)"; head -3 $O/timeline_probe_$n.txt
done
