#!/bin/bash
# round 6, call 24: non-temporal GEMM output stores (VIT_GEMM_NT=1) vs default, B/16 step, same diagnostic binary,
# alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06x; mkdir -p $O
export VITMI_BENCH_TRAIN_EPOCH=0
D=$PWD/vit-of-pytorch_amd/vitmi/diag/libvit_hip.so
for r in 1 2 3; do
  for nt in 0 1; do
    VITMI_LIB=$D VIT_GEMM_NT=$nt timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${nt}_$r.json 2> $O/b_${nt}_$r.err || { tail -5 $O/b_${nt}_$r.err; exit 1; }
    echo "nt=$nt run $r: $(tail -1 $O/b_${nt}_$r.json | grep -o '"value": [0-9.]*' | head -1)"
  done
done
