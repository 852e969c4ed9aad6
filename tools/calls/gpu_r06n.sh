#!/bin/bash
# round 6, call 14: wave-split remainder on 192 x 128 tiles (diagnostic config 12: 216 workgroups for the N = 768
# remainder instead of 324 128^2 ones, one per CU) against the 128^2 default: output digests + timings
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06n; mkdir -p $O
export VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/diag/libvit_hip.so
VIT_GEMM_REM_CFG=0 timeout -k 10 200 python3 -u tools/dbg/rem_check.py > $O/digest_0.txt 2>&1 || { cat $O/digest_0.txt; exit 1; }
VIT_GEMM_REM_CFG=12 timeout -k 10 200 python3 -u tools/dbg/rem_check.py > $O/digest_12.txt 2>&1 || { cat $O/digest_12.txt; exit 1; }
grep -v amdgpu.ids $O/digest_0.txt > $O/d0; grep -v amdgpu.ids $O/digest_12.txt > $O/d12
paste $O/d0 $O/d12
for r in 1 2; do for c in 0 12; do
  echo "== rem cfg $c run $r" >> $O/bench.txt
  VIT_GEMM_REM_CFG=$c timeout -k 10 300 python3 -u tools/gemm_bench.py --tiles 0 --rounds 3 \
    --shapes fc2:4,out:4,qkvdg:1,fc1dg:1,out:1,fc1dgk:1,outk:1,fc2dg:9,fc1:8 >> $O/bench.txt 2>&1 || exit 1
done; done
grep -v amdgpu.ids $O/bench.txt
