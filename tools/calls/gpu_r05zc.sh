#!/bin/bash
# round 5, call 30: the fused cls distillation loss (vit_cls_mse), the approximator's row mask by vit_rows_select and
# the vectorized batched cast, the router mean broadcast in segment_colsum_bcast (ABI 16): kernel + Res-ViT tests, then same-box A/B VITMI_RESVIT_NO_FUSED_DISTILL=1/0
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zc; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_resvit_gpu.py tests/test_resvit_train_gpu.py "tests/test_kernels_gpu.py::test_cast_pad_batch_matches_single_casts" "tests/test_kernels_gpu.py::test_segment_colsum_bcast" "tests/test_kernels_gpu.py::test_segment_colsum_and_router_dx_gate" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    VITMI_RESVIT_NO_FUSED_DISTILL=$v timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 10 --warmup 3 --no-cpu-baseline > $O/nd${v}_$r.json 2> $O/nd${v}_$r.err || { tail -5 $O/nd${v}_$r.err; exit 1; }
    echo "no_fused_distill=$v run $r: $(grep -o '"value": [0-9.]*' $O/nd${v}_$r.json | head -1)"
  done
done
