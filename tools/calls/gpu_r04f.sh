#!/bin/bash
# round 4, call 6: hd-80 attention on 80-wide images (ViT-H/14): attention tests, standalone A/B against the
# HEAD kernels (vitmi/ab: 96-wide images) at H/14 bs 128 and B/16 bs 256, then the H/14 bs 128 step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  echo "base:"; VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/ab/libvit_hip.so timeout -k 10 120 python -u tools/attn_bench.py 128 257 16 80 0 256 197 12 64 0 2>&1 | grep -v amdgpu.ids
  echo "new:"; timeout -k 10 120 python -u tools/attn_bench.py 128 257 16 80 0 256 197 12 64 0 2>&1 | grep -v amdgpu.ids
done
timeout -k 10 300 python3 -u bench.py --arch h14 --batch 128 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_h14.json 2> $O/bench_h14.err || { tail -5 $O/bench_h14.err; exit 1; }
tail -c 400 $O/bench_h14.json
