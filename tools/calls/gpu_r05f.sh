#!/bin/bash
# round 5, call 6: every forward / data-gradient GEMM reads its weight in place (M/N-contiguous B on the half-tile
# ping-pong, no transposed copies): the full GPU suite, then a same-box A/B of the B/16 step against the previous
# commit (abase/, tools/ab_tree.sh 870f926), and the split-K weight gradients on the half-tile kernel
# (VIT_GEMM_SPLITK_CFG=9, diagnostic library) against gemm_pp_kernel (=5)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  (cd abase && timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > ../$O/base_$r.json 2> ../$O/base_$r.err) || { tail -3 $O/base_$r.err; exit 1; }
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/new_$r.json 2> $O/new_$r.err || { tail -3 $O/new_$r.err; exit 1; }
  echo "base $r: $(grep -o '"value": [0-9.]*' $O/base_$r.json | head -1)  new $r: $(grep -o '"value": [0-9.]*' $O/new_$r.json | head -1)"
done
export VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/diag/libvit_hip.so
for r in 1 2; do
  for c in 5 9; do
    VIT_GEMM_SPLITK_CFG=$c timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/sk${c}_$r.json 2> $O/sk${c}_$r.err || { tail -3 $O/sk${c}_$r.err; exit 1; }
    echo "splitk cfg $c run $r: $(grep -o '"value": [0-9.]*' $O/sk${c}_$r.json | head -1)"
  done
done
