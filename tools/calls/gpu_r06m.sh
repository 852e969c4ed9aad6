#!/bin/bash
# round 6, call 13 (v2: wave 7 issues the K / V after a counter spin): attention backward without the stage-1/2 barrier (strip masks, last-reader K/V hand-off,
# extra strip on the idle wave's SIMD): attention tests + parity suite, then kernel A/B against HEAD's kernel
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > $O/tests_attn.log 2>&1 || { tail -30 $O/tests_attn.log; exit 1; }
tail -2 $O/tests_attn.log
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests_parity.log 2>&1 || { tail -30 $O/tests_parity.log; exit 1; }
tail -2 $O/tests_parity.log
for r in 1 2; do
  echo "== new" >> $O/ab.txt
  timeout -k 10 120 python3 -u tools/attn_bench.py 256 197 12 64 0 64 197 16 64 0 128 197 16 80 0 >> $O/ab.txt 2>&1 || exit 1
  echo "== base (HEAD)" >> $O/ab.txt
  VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/ab/libvit_hip.so timeout -k 10 120 python3 -u tools/attn_bench.py 256 197 12 64 0 64 197 16 64 0 128 197 16 80 0 >> $O/ab.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/ab.txt
