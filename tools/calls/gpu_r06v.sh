#!/bin/bash
# round 6, call 22: tile order (VIT_GEMM_GROUP_M) for the split-K weight gradients (diagnostic library)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06v; mkdir -p $O
export VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/diag/libvit_hip.so
python3 -c "import sys; sys.path.insert(0, 'vit-of-pytorch_amd'); from vitmi import _lib; _lib.load()" || exit 1
for r in 1 2; do for gm in 8 1 2 4 16; do
  echo "== group_m $gm run $r" >> $O/gm.txt
  VIT_GEMM_GROUP_M=$gm timeout -k 10 200 python3 -u tools/gemm_bench.py --tiles 0 --rounds 3 --shapes "" --wgrad --splits 7 >> $O/gm.txt 2>&1 || exit 1
done; done
grep -v amdgpu.ids $O/gm.txt
