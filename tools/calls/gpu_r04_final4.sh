#!/bin/bash
# round 4, end of session (after the gradient sinks): the full GPU suite, smoke(), the default bench line (with the CPU baseline) and the
# Res-ViT-B/16 bs 128 line on the final code
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_final_v6; mkdir -p $O
step() { echo "== $1"; shift; "$@" || { echo "FAILED: $*"; exit 1; }; }
step "pytest -m gpu" timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
step "smoke" timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
step "bench" timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_b16.json 2> $O/bench_b16.err
grep -o '"value": [0-9.]*' $O/bench_b16.json | head -1
step "resvit" timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_resvit.json 2> $O/bench_resvit.err
grep -o '"value": [0-9.]*' $O/bench_resvit.json | head -1
