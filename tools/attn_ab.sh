#!/bin/bash
# attention kernel tests + A/B timing (kernel variants; resident vs tiled) in one GPU call
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_submodules_gpu.py -m gpu -q -x --timeout 120 \
    --timeout-method thread -k "attention" > $O/attn_tests.log 2>&1 || { tail -30 $O/attn_tests.log; exit 1; }
tail -2 $O/attn_tests.log
CASES=${CASES:-"256 197 12 64 1  256 197 12 64 2  128 257 16 80 1  64 577 12 64 0"}
echo "== default"; timeout -k 10 120 python -u tools/attn_bench.py $CASES || exit 1
echo "== fwd variant 1 (one-shot lean), bwd round-1"; VIT_ATTN_FWD_VARIANT=1 VIT_ATTN_BWD_VARIANT=2 timeout -k 10 120 \
    python -u tools/attn_bench.py 256 197 12 64 1 || exit 1
