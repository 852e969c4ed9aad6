#!/bin/bash
# round 6, call 17: MFMA priority vs reader priority in gemm_pp2 (VIT_GEMM_PRIO 1 = default: setprio around the MFMA
# cluster, 0 = none, 2 = around the reading group's fragment reads + DMA issue): weight-gradient and forward shapes,
# then slot stamps under each
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06q; mkdir -p $O
export VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/diag/libvit_hip.so
python3 -c "import sys; sys.path.insert(0, \"vit-of-pytorch_amd\"); from vitmi import _lib; _lib.load()" || exit 1
for r in 1 2; do for pr in 1 0 2; do
  echo "== prio $pr run $r" >> $O/bench.txt
  VIT_GEMM_PRIO=$pr timeout -k 10 300 python3 -u tools/gemm_bench.py --tiles 0 --rounds 3 --shapes fc2:4,qkvdg:1,fc1dg:1 --wgrad --splits 7,9 >> $O/bench.txt 2>&1 || exit 1
done; done
grep -v amdgpu.ids $O/bench.txt
for pr in 0 2; do
  echo "== stamps prio $pr" >> $O/stamps.txt
  VIT_GEMM_PRIO=$pr VIT_GEMM_DIAG=4 timeout -k 10 200 python3 -u tools/dbg/pp2_stamps.py >> $O/stamps.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/stamps.txt | grep -A4 "run 1\|== "
