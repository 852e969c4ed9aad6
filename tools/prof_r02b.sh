#!/bin/bash
# Round-2 evidence, second set (after the round's kernel changes): bench line, kernel trace + stats and step
# timeline, per-kernel PMC passes (MFMA busy; FETCH_SIZE; WRITE_SIZE, each its own run) and the per-launch
# HBM traffic JSONs of the two roofline kernels (split-K weight gradient, fc1 forward) that bench.py reads.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02b
V=${V:-3}
mkdir -p $O
step() { echo "== $1"; shift; "$@" || { echo "FAILED: $*"; exit 1; }; }
step "bench b16" timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_b16_v$V.json
step "ktrace" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/ktrace.log 2>&1
S=$(find $O/ktrace -name "*kernel_stats.csv" | head -1)
T=$(find $O/ktrace -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py $S 13 > $O/kernel_summary.txt
python3 tools/trace_step.py $T 1 $O/step_launches.txt > $O/step_timeline.txt
cp $S $O/kernel_stats.csv
step "pmc mfma" timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $O/pmc_mfma -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_mfma.log 2>&1
step "pmc fetch" timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1
step "pmc write" timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1
F=$(find $O/pmc_fetch -name "*counter_collection.csv" | head -1)
W=$(find $O/pmc_write -name "*counter_collection.csv" | head -1)
python3 tools/kernel_pmc.py $O/kernel_pmc.txt $(find $O/pmc_mfma $O/pmc_fetch $O/pmc_write -name "*counter_collection.csv") > /dev/null
python3 tools/pmc_traffic.py "gemm_pp_kernel<256, 64, 2, false, false, 7>" $F $W $O/wgrad_traffic_v1.json > /dev/null
python3 tools/pmc_traffic.py "gemm_pp2_kernel<true, true, 8>|gemm_bf16_kernel<128, 128, 64, 2, 2, 2, true, true, 8>" $F $W $O/fc1_traffic_v1.json > /dev/null
head -22 $O/kernel_summary.txt
head -14 $O/kernel_pmc.txt
tail -c 1500 $O/bench_b16_v$V.json
