#!/bin/bash
# round 5, call 1: the full GPU suite on the round's first changes (build id, Res-ViT advice fixes, bench fields),
# the B/16 bench line with the new roofline_fwd_dgrad block, and a calibration of every forward / data-gradient
# GEMM shape: production dispatch vs the half-tile ping-pong alone (tile 9), its epilogue without global stores
# (VIT_GEMM_DIAG=1) and its main loop alone (=2), and hipBLASLt (torch.matmul) on the same operands
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py > $O/bench_b16.json 2> $O/bench_b16.err || { tail -5 $O/bench_b16.err; exit 1; }
head -c 600 $O/bench_b16.json; echo
SH="fc1:8,fc2:4,outk:4/1,qkvk:2,fc2dgk:9,fc1dgk:1,qkvdg:1"
timeout -k 10 300 python -u tools/gemm_bench.py --tiles 0,9 --shapes $SH --blas > $O/gemm_prod.txt 2>&1 || { tail -5 $O/gemm_prod.txt; exit 1; }
grep -v amdgpu.ids $O/gemm_prod.txt
for d in 1 2; do
  VIT_GEMM_DIAG=$d VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/diag/libvit_hip.so timeout -k 10 300 python -u tools/gemm_bench.py --tiles 9 --shapes $SH > $O/gemm_diag$d.txt 2>&1 || { tail -5 $O/gemm_diag$d.txt; exit 1; }
  echo "diag $d:"; grep -v amdgpu.ids $O/gemm_diag$d.txt
done
