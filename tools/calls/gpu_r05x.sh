#!/bin/bash
# round 5, call 25: the first routed layer's teacher output from the student's layer forward (one layer forward fewer
# per step): Res-ViT tests (reference trajectory, graphed = eager, DP), then same-box A/B VITMI_RESVIT_TEACHER_PASS=1/0
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_resvit_gpu.py tests/test_resvit_train_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for tp in 1 0; do
    VITMI_RESVIT_TEACHER_PASS=$tp timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 10 --warmup 3 --no-cpu-baseline > $O/tp${tp}_$r.json 2> $O/tp${tp}_$r.err || { tail -5 $O/tp${tp}_$r.err; exit 1; }
    echo "teacher_pass=$tp run $r: $(grep -o '"value": [0-9.]*' $O/tp${tp}_$r.json | head -1)"
  done
done
