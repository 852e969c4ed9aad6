#!/bin/bash
# round 4, call 19: persistent attention backward, the last key pair skips its wholly padded second tile
# (stamps of waves 0 and 6, DIAG build), attention tests, same-box A/B against HEAD (vitmi/ab),
# then B/16 bench lines (new, base) for the step effect
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04r; mkdir -p $O
VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/diag/w6/libvit_hip.so timeout -k 10 120 python -u tools/attn_stamps.py 2>&1 | grep "wave . item" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  echo "base:"; VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/ab/libvit_hip.so timeout -k 10 120 python -u tools/attn_bench.py 256 197 12 64 0 64 197 16 64 0 2>&1 | grep bwd
  echo "new:"; timeout -k 10 120 python -u tools/attn_bench.py 256 197 12 64 0 64 197 16 64 0 2>&1 | grep bwd
done
for r in 1 2; do
  VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/ab/libvit_hip.so timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/base_$r.json 2> $O/base_$r.err || { tail -3 $O/base_$r.err; exit 1; }
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/new_$r.json 2> $O/new_$r.err || { tail -3 $O/new_$r.err; exit 1; }
  echo "base $r: $(grep -o '"value": [0-9.]*' $O/base_$r.json | head -1)  new $r: $(grep -o '"value": [0-9.]*' $O/new_$r.json | head -1)"
done
