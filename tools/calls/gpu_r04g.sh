#!/bin/bash
# round 4, call 7: DPP column sums in the two-stage attention backward (bias partials), the graphed Res-ViT step:
# attention + Res-ViT GPU tests, hd-80 phase stamps with bias partials, attention micro-bench, Res-ViT bs 128 bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_resvit_train_gpu.py -k "attention or resvit or graphed or adamw or flat" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/diag/libvit_hip.so timeout -k 10 100 python tools/attn2_stamps.py 128 257 16 80 bias 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python -u tools/attn_bench.py 128 257 16 80 0 256 197 12 64 0 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_resvit.json 2> $O/bench_resvit.err || { tail -5 $O/bench_resvit.err; exit 1; }
tail -c 600 $O/bench_resvit.json
