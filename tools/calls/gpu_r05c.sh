#!/bin/bash
# round 5, call 3: the ping-pong GEMM with 32-deep k-tiles (diagnostic configs 10: same ring, 11: a ring three
# 32-deep k-tiles ahead) against config 9 (64-deep): bit-exactness, whole kernel and main loop alone
# (VIT_GEMM_DIAG=2) on the B/16 shapes; the production library's GEMM tests (generalised ring code, wave split
# with column partials)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
export VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/diag/libvit_hip.so
timeout -k 10 120 python -u tools/gemm_cfg_check.py 10,11 > $O/cfg_check.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/cfg_check.txt; [ $rc -eq 0 ] || exit $rc
SH="fc1:8,fc2:4,outk:1,qkvk:2,fc2dgk:9,fc1dgk:1,qkvdg:1"
timeout -k 10 400 python -u tools/gemm_bench.py --tiles 9,10,11 --shapes $SH > $O/full.txt 2>&1 || { tail -5 $O/full.txt; exit 1; }
grep -v amdgpu.ids $O/full.txt
VIT_GEMM_DIAG=2 timeout -k 10 400 python -u tools/gemm_bench.py --tiles 9,10,11 --shapes $SH > $O/main.txt 2>&1 || { tail -5 $O/main.txt; exit 1; }
echo "main loop only:"; grep -v amdgpu.ids $O/main.txt
