#!/bin/bash
# attention iteration: debug errors, kernel tests, micro-bench, stamps, parity + step A/B vs ./abase
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/attn; mkdir -p $O
timeout -k 10 100 python -u tools/attn_dbg.py > $O/dbg.txt 2>&1 || { tail -5 $O/dbg.txt; exit 1; }
grep -v amdgpu $O/dbg.txt | cut -c1-150
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/attn_bench.py 256 197 12 64 0 > $O/new.txt 2>&1 || { tail -5 $O/new.txt; exit 1; }
ATTN_QROWS=1 timeout -k 10 120 python -u tools/attn_bench.py 256 197 12 64 0 > $O/new_q1.txt 2>&1 || { tail -5 $O/new_q1.txt; exit 1; }
grep bwd $O/new.txt $O/new_q1.txt
VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/ab/libvit_hip.so timeout -k 10 120 python tools/attn_stamps.py 2>&1 | grep wave
if [ -n "$1" ]; then bash tools/gpu_ab.sh "$1" 2; fi
