#!/bin/bash
# round 6, call 15: gemm_pp2 slot timeline from in-kernel stamps (diagnostic library, VIT_GEMM_DIAG=4)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06o; mkdir -p $O
export VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/diag/libvit_hip.so
VIT_GEMM_DIAG=4 timeout -k 10 200 python3 -u tools/dbg/pp2_stamps.py > $O/stamps.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/stamps.txt
exit $rc
