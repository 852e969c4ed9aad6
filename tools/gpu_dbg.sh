#!/bin/bash
# attention tests after the variant cleanup; A/B: s_setprio around the ping-pong GEMM MFMA clusters
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread -k "attention" > gpurun_out/t_dbg.log 2>&1
rc=$?; echo "attn tests rc=$rc $(tail -1 gpurun_out/t_dbg.log)"; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
for v in 0 1; do
VIT_GEMM_PRIO=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_ab.log 2>&1 || { tail -5 gpurun_out/b_ab.log; exit 1; }
echo "prio=$v $(tail -1 gpurun_out/b_ab.log | grep -o '"value": [0-9.]*') $(tail -1 gpurun_out/b_ab.log | grep -o '"frac": [0-9.]*' | head -1)"
done
done
