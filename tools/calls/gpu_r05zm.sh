#!/bin/bash
# round 5, call 41: the teacher pass writes only GELU(u) of fc1 (C == C2 in the fused layer without a backward); A/B
# VITMI_RESVIT_TEACHER_DGELU=1/0 after the kernel and Res-ViT tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zm; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_resvit_gpu.py tests/test_resvit_train_gpu.py "tests/test_kernels_gpu.py::test_gelu_dgelu_same_buffer_keeps_gelu" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    VITMI_RESVIT_TEACHER_DGELU=$v timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 10 --warmup 3 --no-cpu-baseline > $O/td${v}_$r.json 2> $O/td${v}_$r.err || { tail -5 $O/td${v}_$r.err; exit 1; }
    echo "teacher_dgelu=$v run $r: $(grep -o '"value": [0-9.]*' $O/td${v}_$r.json | head -1)"
  done
done
