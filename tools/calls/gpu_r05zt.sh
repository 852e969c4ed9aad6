#!/bin/bash
# round 5, call 48: vit_colsum's chunk loop unrolled per input type (eight loads in flight): kernel, parity and Res-ViT
# tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zt; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_resvit_gpu.py tests/test_resvit_train_gpu.py tests/test_submodules_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
