#!/bin/bash
# round 5, call 27: the distillation loss's cls rows through cls_tap (gradient added in place) and the final LayerNorm on
# the cls rows only: Res-ViT tests, then same-box A/B VITMI_RESVIT_NO_CLS_TAP=1/0
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05z; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_resvit_gpu.py tests/test_resvit_train_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    VITMI_RESVIT_NO_CLS_TAP=$v timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 10 --warmup 3 --no-cpu-baseline > $O/nt${v}_$r.json 2> $O/nt${v}_$r.err || { tail -5 $O/nt${v}_$r.err; exit 1; }
    echo "no_cls_tap=$v run $r: $(grep -o '"value": [0-9.]*' $O/nt${v}_$r.json | head -1)"
  done
done
