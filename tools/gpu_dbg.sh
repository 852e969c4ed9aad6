#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_resvit_train_gpu.py -v --timeout 200 --timeout-method thread > gpurun_out/t_dbg.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E " gpurun_out/t_dbg.log | cut -c1-600 | head -40; exit $rc
