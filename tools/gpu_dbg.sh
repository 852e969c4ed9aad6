#!/bin/bash
# LayerNorm fusion ceiling: the step with the per-layer LayerNorm forward / backward launches skipped
set -o pipefail
export TMPDIR=/tmp
for i in 1 2; do
for v in none fwd bwd fwdbwd; do
VITMI_DIAG_SKIP_LN=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_ab.log 2>&1 || { tail -5 gpurun_out/b_ab.log; exit 1; }
echo "skip_ln=$v $(tail -1 gpurun_out/b_ab.log | grep -o '"value": [0-9.]*') $(tail -1 gpurun_out/b_ab.log | grep -o '"ms_per_step": [0-9.]*')"
done
done
