#!/bin/bash
# rocprofv3 kernel trace + stats of one command; prints the top kernels (tools/prof_summary.py).
#   usage: bash tools/kstats.sh TAG python3 tools/attn_bench.py ...
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/ks_$TAG
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- "$@" > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
S=$(find $O -name "*kernel_stats.csv" | head -1)
python3 tools/prof_summary.py $S 1 | head -${TOP:-20}
