#!/bin/bash
# end-of-session check: full GPU test suite, then the round-2 evidence set (tools/prof_r02b.sh, V=6)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?; tail -2 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
V=6 bash tools/prof_r02b.sh > gpurun_out/prof_v6.log 2>&1
