#!/bin/bash
# round 4, call 3: the persistent GEMM (config 10): its tests, the GEMM kernel tests, a GEMM sweep of the
# B/16 shapes (auto / one-shot 9 / persistent 10), then the default bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_ps_gpu.py -x -v --timeout 200 --timeout-method thread > $O/ps_tests.log 2>&1
rc=$?; tail -25 $O/ps_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_bench.py --tiles 0,9,10 --rounds 3 \
  --shapes fc1:8,qkvk:2,fc2dgk:9,fc1dgk:1,qkvdg:1,outk:1,fc2:1 > $O/gemm_ps.txt 2>&1 || { cat $O/gemm_ps.txt; exit 1; }
cat $O/gemm_ps.txt
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
