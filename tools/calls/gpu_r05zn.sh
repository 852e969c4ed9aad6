#!/bin/bash
# round 5, call 42: the token embedding as one GEMM with the PATCH epilogue (vitmi.resvit_fused.embed_tokens); A/B
# VITMI_RESVIT_NO_FUSED_EMBED=1/0 after the kernel and Res-ViT tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zn; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_resvit_gpu.py tests/test_resvit_train_gpu.py "tests/test_kernels_gpu.py::test_im2col_and_embed_grad" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    VITMI_RESVIT_NO_FUSED_EMBED=$v timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 10 --warmup 3 --no-cpu-baseline > $O/ne${v}_$r.json 2> $O/ne${v}_$r.err || { tail -5 $O/ne${v}_$r.err; exit 1; }
    echo "no_fused_embed=$v run $r: $(grep -o '"value": [0-9.]*' $O/ne${v}_$r.json | head -1)"
  done
done
