#!/bin/bash
# round 6, call 3: w4 prototype ablations (no global loads / no image writes / no fragment reads / MFMA only)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c; mkdir -p $O
step() { echo "== $1"; shift; "$@" || { echo "FAILED: $*"; exit 1; }; }
for sh in "50432 768 3072" "50432 768 2304"; do
  W4_DIAG=1 step "proto $sh" timeout -k 10 120 tools/w4_proto $sh >> $O/proto.txt 2>&1
done
grep -v "rel fro" $O/proto.txt
step "sgd dev test" timeout -k 10 300 python -u -m pytest tests/test_optim_dev_gpu.py -x -q --timeout 120 --timeout-method thread > $O/sgd_test.log 2>&1
tail -3 $O/sgd_test.log
