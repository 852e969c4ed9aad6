#!/bin/bash
# GEMM epilogue probe (profiles/r02/gemm_epilogue_diag.txt): VIT_GEMM_DIAG 0 = full kernel,
# 1 = no global stores (generic epilogue), 2 = main loop only.
set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k gemm 2>&1 | tail -3
for d in 0 1 2; do
  echo "== VIT_GEMM_DIAG=$d"
  VIT_GEMM_DIAG=$d timeout -k 10 120 python -u tools/gemm_bench.py --tiles 9 --shapes fc1:8,fc2:4,out:4,fc2dgk:9,qkvk:2,fc1dgk:1 --rounds 3
done
echo "== split-K weight gradients (tile 5, split 8 and the one-wave split)"
timeout -k 10 120 python -u tools/gemm_bench.py --tiles 5 --shapes "" --wgrad --splits 7,8 --rounds 1
