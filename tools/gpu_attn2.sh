#!/bin/bash
# attention backward iteration: kernel tests, micro-bench (this tree vs ./abase), stamps of the diagnostic build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/attn; mkdir -p $O
timeout -k 10 100 python -u tools/attn_dbg.py && timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/attn_bench.py 256 197 12 64 0 > $O/new.txt 2>&1 || { tail -5 $O/new.txt; exit 1; }
ATTN_QROWS=1 timeout -k 10 120 python -u tools/attn_bench.py 256 197 12 64 0 > $O/new_q1.txt 2>&1 || { tail -5 $O/new_q1.txt; exit 1; }
grep bwd $O/new.txt $O/new_q1.txt
VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/ab/libvit_hip.so timeout -k 10 120 python tools/attn_stamps.py
