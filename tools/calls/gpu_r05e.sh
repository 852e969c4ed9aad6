#!/bin/bash
# round 5, call 5: the half-tile ping-pong (config 9) with inline-asm transposed fragment reads for M/N-contiguous
# operands and the XCD-major split-K remap: GEMM tests, then the split-K weight gradients on it against
# gemm_pp_kernel (config 5, today's), and the data gradients with the weights as they are (M/N-contiguous B)
# against the K-contiguous transposed copies
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/gemm_bench.py --shapes "" --wgrad --tiles 5,9 --splits 5,7,9,14 > $O/wgrad.txt 2>&1 || { tail -5 $O/wgrad.txt; exit 1; }
grep -v amdgpu.ids $O/wgrad.txt
timeout -k 10 400 python -u tools/gemm_bench.py --tiles 0,3,5,9 --shapes "fc2dg:9,fc2dgk:9,fc1dg:1,fc1dgk:1,qkv:2,qkvk:2,out:1,outk:1" > $O/mn.txt 2>&1 || { tail -5 $O/mn.txt; exit 1; }
grep -v amdgpu.ids $O/mn.txt
