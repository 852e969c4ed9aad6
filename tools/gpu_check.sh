#!/bin/bash
# One gpurun call: GPU tests, bench line, GEMM tile comparison. Every GPU step has its own time
# limit and the steps are chained: the first failure ends the call.
#   usage: bash tools/gpu_check.sh [tests] [bench] [gemm] [prof]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
want() { [ $# -eq 0 ] || [[ " $ARGS " == *" $1 "* ]]; }
ARGS="$*"
[ -z "$ARGS" ] && ARGS="tests bench gemm"
if [[ " $ARGS " == *" tests "* ]]; then
  echo "== pytest -m gpu" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
      --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
fi
if [[ " $ARGS " == *" gemm "* ]]; then
  echo "== gemm tiles" && timeout -k 10 400 python -u tools/gemm_bench.py --tiles ${TILES:-3,5,6} --epis ${EPIS:-1,3} \
      --blas > $O/gemm_bench.log 2>&1 || { tail -20 $O/gemm_bench.log; exit 1; }
  cat $O/gemm_bench.log
fi
if [[ " $ARGS " == *" bench "* ]]; then
  echo "== bench" && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 \
      || { tail -20 $O/bench.log; exit 1; }
  tail -1 $O/bench.log
fi
if [[ " $ARGS " == *" prof "* ]]; then
  echo "== rocprofv3 kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_prof.log 2>&1 \
      || { tail -20 $O/bench_prof.log; exit 1; }
  find $O/prof -name "*kernel_stats.csv" | head -3
fi
exit 0
