#!/bin/bash
# Profiling recipe for the bench step (MI355X_MICROARCH.md, HBM / rocprofv3 sections):
#   1. kernel trace + stats of the default bench (per-kernel averages; the fc1 GEMM average must
#      agree with bench.py's live HIP-event roofline number),
#   2. FETCH_SIZE and WRITE_SIZE in separate --pmc passes, restricted to the bench's roofline kernel
#      (the fc1 forward GEMM, EPI_BIAS_GELU instantiation), for roofline.traffic.
# usage: bash tools/prof.sh TAG     (outputs under gpurun_out/prof_TAG)
set -e
export TMPDIR=/tmp
TAG=${1:-cur}
O=gpurun_out/prof_$TAG
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_ktrace.log 2>&1
S=$(find $O/ktrace -name "*kernel_stats.csv" | head -1)
python3 tools/prof_summary.py $S 13 > $O/summary.txt
RX=${ROOF_RX:-'gemm_\w+_kernel<.*, 8>'}
timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/fetch -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_fetch.log 2>&1
timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/write -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_write.log 2>&1
python3 tools/pmc_traffic.py "$RX" $(find $O/fetch -name "*counter_collection.csv" | head -1) \
    $(find $O/write -name "*counter_collection.csv" | head -1) $O/traffic.json > /dev/null
cat $O/summary.txt | head -30
cat $O/traffic.json
