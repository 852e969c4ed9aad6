#!/bin/bash
# end-of-session check: the whole -m gpu suite, smoke(), one default bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -3 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -3 $O/bench.err; exit 1; }
head -c 300 $O/bench.json; echo
