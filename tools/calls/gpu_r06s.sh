#!/bin/bash
# round 6, call 19: the B/16 bs-256 step with the weight gradients' interleaved read slot (auto) vs off, same
# diagnostic binary (VIT_GEMM_ILV unset / 0), alternating, then the production library once
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s; mkdir -p $O
export VITMI_BENCH_TRAIN_EPOCH=0
D=$PWD/vit-of-pytorch_amd/vitmi/diag/libvit_hip.so
for r in 1 2 3; do
  for il in -1 0; do
    VITMI_LIB=$D VIT_GEMM_ILV=$il timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_${il}_$r.json 2> $O/b_${il}_$r.err || { tail -5 $O/b_${il}_$r.err; exit 1; }
    echo "ilv=$il run $r: $(tail -1 $O/b_${il}_$r.json | grep -o '"value": [0-9.]*' | head -1)"
  done
done
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_prod.json 2> $O/b_prod.err || { tail -5 $O/b_prod.err; exit 1; }
echo "production: $(tail -1 $O/b_prod.json | grep -o '"value": [0-9.]*' | head -1)"
