#!/bin/bash
# round 6, call 18: gemm_pp2 read slot with the LDS-DMA pieces interleaved between the fragment reads
# (VIT_GEMM_ILV=1) against reads-then-DMA (0): output digests, timings (forward / dgrad / weight-gradient shapes),
# slot stamps
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06r; mkdir -p $O
export VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/diag/libvit_hip.so
python3 -c "import sys; sys.path.insert(0, 'vit-of-pytorch_amd'); from vitmi import _lib; _lib.load()" || exit 1
VIT_GEMM_ILV=0 timeout -k 10 200 python3 -u tools/dbg/rem_check.py > $O/digest_0.txt 2>&1 || { cat $O/digest_0.txt; exit 1; }
VIT_GEMM_ILV=1 timeout -k 10 200 python3 -u tools/dbg/rem_check.py > $O/digest_1.txt 2>&1 || { cat $O/digest_1.txt; exit 1; }
grep -v amdgpu.ids $O/digest_0.txt > $O/d0; grep -v amdgpu.ids $O/digest_1.txt > $O/d1
paste $O/d0 $O/d1
cmp -s $O/d0 $O/d1 || { echo "DIGESTS DIFFER"; exit 1; }
for r in 1 2; do for il in 0 1; do
  echo "== ilv $il run $r" >> $O/bench.txt
  VIT_GEMM_ILV=$il timeout -k 10 300 python3 -u tools/gemm_bench.py --tiles 0 --rounds 3 --shapes fc2:4,fc1:8,qkvdg:1,fc1dg:1,fc2dg:9 --wgrad --splits 7,9 >> $O/bench.txt 2>&1 || exit 1
done; done
grep -v amdgpu.ids $O/bench.txt
VIT_GEMM_ILV=1 VIT_GEMM_DIAG=4 timeout -k 10 200 python3 -u tools/dbg/pp2_stamps.py > $O/stamps.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/stamps.txt | grep -A4 "run 1"
