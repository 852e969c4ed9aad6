#!/bin/bash
# round 4, call 25: row-pipelined LayerNorm forward (each wave walks rows, next row's loads in flight, at most 2048
# blocks): LayerNorm / parity tests, ln_bench A/B against HEAD's kernel (vitmi/ab), then B/16 bench lines, same box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04y2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py -k "layernorm or ln_ or b16_full or step_matches or exact" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  echo "base:"; VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/ab/libvit_hip.so timeout -k 10 120 python -u tools/ln_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
  echo "new:"; timeout -k 10 120 python -u tools/ln_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
for r in 1 2; do
  VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/ab/libvit_hip.so timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/base_$r.json 2> $O/base_$r.err || { tail -3 $O/base_$r.err; exit 1; }
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/new_$r.json 2> $O/new_$r.err || { tail -3 $O/new_$r.err; exit 1; }
  echo "base $r: $(grep -o '"value": [0-9.]*' $O/base_$r.json | head -1)  new $r: $(grep -o '"value": [0-9.]*' $O/new_$r.json | head -1)"
done
