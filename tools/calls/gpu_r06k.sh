#!/bin/bash
# round 6, call 11: the 8-phase GEMM schedule (diagnostic tile config 12) against gemm_pp2 (config 9): parity + timing
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06k; mkdir -p $O
export VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/diag/libvit_hip.so
timeout -k 10 240 python3 -u tools/dbg/ph8_check.py > $O/ph8.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/ph8.txt
exit $rc
