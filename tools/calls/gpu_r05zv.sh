#!/bin/bash
# round 5, call 50: vit_segment_colsum with eight rows in flight per lane: kernel + Res-ViT tests, kernel stats and a
# Res-ViT A/B against abase (HEAD before the change)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zv; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_resvit_gpu.py tests/test_resvit_train_gpu.py "tests/test_kernels_gpu.py::test_segment_colsum_bcast" "tests/test_kernels_gpu.py::test_segment_colsum_and_router_dx_gate" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for t in abase .; do
  n=$(basename $t)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$n -o run -- python3 $t/bench.py --arch resvit_b16 --steps 4 --warmup 2 --no-cpu-baseline > $O/kt_$n.log 2>&1 || { tail -5 $O/kt_$n.log; exit 1; }
  S=$(find $O/kt_$n -name "*kernel_stats.csv" | head -1)
  echo "$t:"; grep -E "segment_colsum" $S | cut -d, -f1-4
  rm -rf $O/kt_$n
done
for r in 1 2; do
  for t in abase .; do
    timeout -k 10 300 python3 -u $t/bench.py --arch resvit_b16 --steps 10 --warmup 3 --no-cpu-baseline > $O/rv_$(basename $t)_$r.json 2> $O/rv_$(basename $t)_$r.err || { tail -5 $O/rv_$(basename $t)_$r.err; exit 1; }
    echo "$t run $r: $(grep -o '"value": [0-9.]*' $O/rv_$(basename $t)_$r.json | head -1)"
  done
done
