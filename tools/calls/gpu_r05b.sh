#!/bin/bash
# round 5, call 2: can the ping-pong main loop absorb its epilogue's stores? (tools/overlap_bench: LDS-DMA fills +
# fragment reads + MFMAs per half k-tile, with 0 .. 1.5x fc1's store rate issued behind the DMA); and which
# hipBLASLt kernels beat our main loop on the N = 768 shapes (kernel names from a rocprofv3 kernel trace)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 120 ./tools/overlap_bench > $O/overlap_bench.txt 2>&1 || { tail -5 $O/overlap_bench.txt; exit 1; }
cat $O/overlap_bench.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/blas -o blas -- python3 tools/gemm_bench.py --tiles 9 --shapes qkvdg:1,fc1dgk:1,outk:1,fc2:1 --blas --rounds 1 > $O/blas.log 2>&1 || { tail -5 $O/blas.log; exit 1; }
find $O/blas -name "*stats*" | head
f=$(find $O/blas -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -c1-220 "$f" | head -20
