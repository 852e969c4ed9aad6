#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -x -q --timeout 150 --timeout-method thread -k "attention or c1 or trajectory" > gpurun_out/t_dbg2.log 2>&1
echo "rc=$? $(tail -1 gpurun_out/t_dbg2.log)"
