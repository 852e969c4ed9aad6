#!/bin/bash
# round 6, call 12: persistent row-panel GEMM (diagnostic tile config 12: 197 workgroups x 3 column tiles at
# N = 768) against the production call (tile 0: one-shot half-tile kernel + 128^2 wave-split remainder) and config 9
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06l; mkdir -p $O
export VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/diag/libvit_hip.so
timeout -k 10 240 python3 -u tools/dbg/panel_check.py > $O/panel_check.txt 2>&1 || { grep -v amdgpu.ids $O/panel_check.txt; exit 1; }
grep -v amdgpu.ids $O/panel_check.txt
timeout -k 10 300 python3 -u tools/gemm_bench.py --tiles 0,9,12 --rounds 5 \
  --shapes fc2:4,out:4,qkvdg:1,fc1dg:1,outk:1,fc1dgk:1 > $O/panel_bench.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/panel_bench.txt
exit $rc
