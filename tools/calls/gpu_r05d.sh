#!/bin/bash
# round 5, call 4: which tile config should run the wave-split remainder rows (VIT_GEMM_REM_CFG, diagnostic
# library): 0 = 128x128x64 (today), 2 = 256x128x64 1 WG/CU, 3 = 256x128x32 2 WG/CU, 4 = 128x128x32 4-stage,
# 6 = 256x128 ping-pong, on the production dispatch (tile 0) of the B/16 shapes with a remainder
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05d; mkdir -p $O
export VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/diag/libvit_hip.so
SH="fc2:4,outk:4/1,fc1dgk:1,qkvdg:1,fc1:8,fc2dgk:9"
for r in 0 2 3 4 6; do
  VIT_GEMM_REM_CFG=$r timeout -k 10 300 python -u tools/gemm_bench.py --tiles 0 --shapes $SH --rounds 5 > $O/rem$r.txt 2>&1 || { tail -5 $O/rem$r.txt; exit 1; }
  echo "rem cfg $r:"; grep -v amdgpu.ids $O/rem$r.txt
done
