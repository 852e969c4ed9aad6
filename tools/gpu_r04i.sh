#!/bin/bash
# round 4, call 9: the 16-wave hd-80 attention backward: attention tests, phase stamps (with bias partials),
# same-box A/B against the committed 8-wave kernel (vitmi/ab), then the H/14 bs 128 step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/diag/libvit_hip.so timeout -k 10 100 python tools/attn2_stamps.py 128 257 16 80 bias 2>&1 | grep -v amdgpu.ids
for r in 1 2; do
  echo "base:"; VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/ab/libvit_hip.so timeout -k 10 120 python -u tools/attn_bench.py 128 257 16 80 0 2>&1 | grep bwd
  echo "new:"; timeout -k 10 120 python -u tools/attn_bench.py 128 257 16 80 0 2>&1 | grep bwd
done
timeout -k 10 300 python3 -u bench.py --arch h14 --batch 128 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_h14.json 2> $O/bench_h14.err || { tail -5 $O/bench_h14.err; exit 1; }
grep -o '"value": [0-9.]*' $O/bench_h14.json | head -1
