#!/bin/bash
# round 4, call 8: graphed Res-ViT step captured on its warm-up stream (tests + bs 128 bench, eager line beside it),
# then a same-box A/B of B/16 bs 256 with the weight-gradient GEMMs on a side stream (VITMI_OVERLAP=1) vs serial
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_resvit_train_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_resvit.json 2> $O/bench_resvit.err || { tail -5 $O/bench_resvit.err; exit 1; }
tail -c 700 $O/bench_resvit.json; echo
for r in 1 2; do
  for ov in 0 1; do
    VITMI_OVERLAP=$ov timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b16_ov${ov}_$r.json 2> $O/b16_ov${ov}_$r.err || { tail -5 $O/b16_ov${ov}_$r.err; exit 1; }
    echo "overlap=$ov run $r: $(grep -o '"value": [0-9.]*' $O/b16_ov${ov}_$r.json | head -1)"
  done
done
