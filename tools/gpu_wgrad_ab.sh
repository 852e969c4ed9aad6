#!/bin/bash
# split-K weight-gradient GEMM change: stamps + standalone timings, GEMM / step tests, bench A/B vs ./abase
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/wg; mkdir -p $O
timeout -k 10 60 tools/gdiag_bin 3072 768 50432 5 7 3 1 1 7 > $O/st.txt 2>&1 || { cat $O/st.txt; exit 1; }
python tools/diag_slots.py $O/st.txt | head -9
timeout -k 10 60 tools/gdiag_bin 2304 768 50432 5 7 -1 1 1 9 | head -1
timeout -k 10 60 tools/gdiag_bin 768 768 50432 5 7 -1 1 1 28 | head -1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh "" 2
