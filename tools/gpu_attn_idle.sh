#!/bin/bash
# attention backward, next-item DMA from the idle stage-2 wave: attention tests, micro-bench, step A/B vs ./abase
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/aidle; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/attn_bench.py 256 197 12 64 0 > $O/new.txt 2>&1 || { tail -5 $O/new.txt; exit 1; }
(cd abase && timeout -k 10 120 python -u tools/attn_bench.py 256 197 12 64 0) > $O/base.txt 2>&1 || { tail -5 $O/base.txt; exit 1; }
grep bwd $O/base.txt $O/new.txt
bash tools/gpu_ab.sh "" 2
