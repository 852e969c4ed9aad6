#!/bin/bash
# round 4, call 4: persistent GEMM v2 (late stores for one-word epilogues, K-split only for K >= 2048)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_ps_gpu.py -x -q --timeout 200 --timeout-method thread > $O/ps_tests.log 2>&1
rc=$?; tail -3 $O/ps_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_bench.py --tiles 0,9,10 --rounds 3 \
  --shapes fc1:8,qkvk:2,fc2dgk:9,fc1dgk:1,qkvdg:1,outk:1,fc2:1 > $O/gemm_ps.txt 2>&1 || { cat $O/gemm_ps.txt; exit 1; }
cat $O/gemm_ps.txt
