#!/bin/bash
# round 5, call 38: the fused layer's output gradient cast on its active rows only (vit_cast_rows_masked, ABI 18) and the
# four-token router_select: kernel + Res-ViT tests, then same-box A/B against abase (HEAD 1941786)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zj; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_resvit_gpu.py tests/test_resvit_train_gpu.py "tests/test_kernels_gpu.py::test_cast_rows_masked" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for t in abase .; do
    timeout -k 10 300 python3 -u $t/bench.py --arch resvit_b16 --steps 10 --warmup 3 --no-cpu-baseline > $O/rv_$(basename $t)_$r.json 2> $O/rv_$(basename $t)_$r.err || { tail -5 $O/rv_$(basename $t)_$r.err; exit 1; }
    echo "$t run $r: $(grep -o '"value": [0-9.]*' $O/rv_$(basename $t)_$r.json | head -1)"
  done
done
