#!/bin/bash
# Round-1 profiling recipe: kernel trace + stats of the default bench, then FETCH_SIZE / WRITE_SIZE passes
# (separate runs, --kernel-trace only alongside) restricted to the GEMM kernels.
set -e
export TMPDIR=/tmp
O=gpurun_out/prof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_ktrace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gemm_bf16_kernel --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex gemm_bf16_kernel --output-format csv -d $O/write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_write.log 2>&1
find $O -name "*.csv" | head -20
