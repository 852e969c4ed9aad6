#!/bin/bash
# attention A/B: attention kernel tests, micro-bench of ./abase vs this tree, then the step bench A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/attn; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u abase/tools/attn_bench.py 256 197 12 64 0 > $O/base.txt 2>&1 || cp tools/attn_bench.py /tmp/ab.py
timeout -k 10 120 python -u tools/attn_bench.py 256 197 12 64 0 > $O/new.txt 2>&1 || { tail -5 $O/new.txt; exit 1; }
ATTN_QROWS=1 timeout -k 10 120 python -u tools/attn_bench.py 256 197 12 64 0 > $O/new_q1.txt 2>&1 || { tail -5 $O/new_q1.txt; exit 1; }
cat $O/base.txt $O/new.txt $O/new_q1.txt
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_submodules_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests2.log 2>&1
rc=$?; tail -2 $O/tests2.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh "" 2
