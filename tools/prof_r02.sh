#!/bin/bash
# Round-2 evidence for profiles/r02/: bench lines (B/16 default, L/16 bs 64, H/14 bs 128), the B/16 step's
# kernel trace + stats, and per-kernel PMC passes (MFMA busy; FETCH_SIZE; WRITE_SIZE, each its own run).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02
mkdir -p $O
step() { echo "== $1"; shift; "$@" || { echo "FAILED: $*"; exit 1; }; }
step "bench b16" timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_b16.json
step "bench l16" timeout -k 10 300 python3 -u bench.py --arch l16 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_l16_bs64.json
step "bench h14" timeout -k 10 300 python3 -u bench.py --arch h14 --batch 128 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_h14_bs128.json
step "ktrace" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/ktrace.log 2>&1
S=$(find $O/ktrace -name "*kernel_stats.csv" | head -1)
python3 tools/prof_summary.py $S 13 > $O/kernel_summary.txt
step "pmc mfma" timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $O/pmc_mfma -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_mfma.log 2>&1
step "pmc fetch" timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1
step "pmc write" timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1
python3 tools/kernel_pmc.py $O/kernel_pmc.txt $(find $O/pmc_mfma $O/pmc_fetch $O/pmc_write -name "*counter_collection.csv")
head -25 $O/kernel_summary.txt
tail -c 600 $O/bench_b16.json; echo; tail -c 400 $O/bench_l16_bs64.json; echo; tail -c 400 $O/bench_h14_bs128.json
