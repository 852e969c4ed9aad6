#!/bin/bash
# round 3: new Res-ViT training-step tests, launcher tests, then the Res-ViT bench line
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_resvit_train_gpu.py tests/test_train_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_r03a.log 2>&1
rc=$?; tail -3 gpurun_out/t_r03a.log
timeout -k 10 300 python -u bench.py --arch resvit_b16 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b_resvit.log 2>&1 || { tail -5 gpurun_out/b_resvit.log; exit 1; }
tail -1 gpurun_out/b_resvit.log | cut -c1-400
exit $rc
