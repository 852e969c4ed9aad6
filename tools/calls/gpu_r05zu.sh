#!/bin/bash
# round 5, call 49: the long bias-gradient column sums (attention backward's per-wave rows) pre-reduced over row chunks
# (engine _BiasReducer, VITMI_COLSUM_SPLIT_MIN): parity / training tests, then same-box B/16 A/B (0 = off)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zu; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_train_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in 0 1024; do
    VITMI_COLSUM_SPLIT_MIN=$v timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b16_${v}_$r.json 2> $O/b16_${v}_$r.err || { tail -5 $O/b16_${v}_$r.err; exit 1; }
    echo "split_min=$v run $r: $(grep -o '"value": [0-9.]*' $O/b16_${v}_$r.json | head -1)"
  done
done
