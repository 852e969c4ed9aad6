#!/bin/bash
# round 6, call 8: GEMM tile-order (VIT_GEMM_GROUP_M) and MFMA-priority (VIT_GEMM_PRIO) knobs re-checked on real
# (random) operands with the diagnostic library, the step's forward / data-gradient shapes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06h; mkdir -p $O
export VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/diag/libvit_hip.so
SH=fc1:8,fc2:4,qkv:2,out:4,fc2dg:9,fc1dg:1,qkvdg:1,out:1
for gm in 8 4 16; do for pr in 1 0; do
  echo "== group_m $gm prio $pr" >> $O/knobs.txt
  VIT_GEMM_GROUP_M=$gm VIT_GEMM_PRIO=$pr timeout -k 10 200 python3 -u tools/gemm_bench.py --tiles 0 --rounds 3 --shapes $SH >> $O/knobs.txt 2>&1 || { echo FAILED; exit 1; }
done; done
grep -v amdgpu.ids $O/knobs.txt
