#!/bin/bash
# round 5, call 44: the batched column sums with 64 row lanes (1024-thread workgroups): kernel tests, then B/16 and
# Res-ViT A/B against abase (HEAD before the change)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zp; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for t in abase .; do
    timeout -k 10 300 python3 -u $t/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b16_$(basename $t)_$r.json 2> $O/b16_$(basename $t)_$r.err || { tail -5 $O/b16_$(basename $t)_$r.err; exit 1; }
    echo "b16 $t run $r: $(grep -o '"value": [0-9.]*' $O/b16_$(basename $t)_$r.json | head -1)"
  done
done
