#!/bin/bash
# round 5, call 51: end-of-round validation v4 on the final tree (after the router_select guard and the vit_colsum unroll): full -m gpu suite, smoke, B/16 bench line (with the CPU
# baseline), Res-ViT-B/16 bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_final_v4; mkdir -p $O
step() { echo "== $1"; shift; "$@" || { echo "FAILED: $*"; exit 1; }; }
step "pytest -m gpu" timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
step "smoke" timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
step "bench b16" timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_b16.json 2> $O/bench_b16.err
tail -c 300 $O/bench_b16.json; echo
step "bench resvit" timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 20 --warmup 5 > $O/bench_resvit_b16.json 2> $O/bench_resvit_b16.err
tail -c 300 $O/bench_resvit_b16.json; echo
