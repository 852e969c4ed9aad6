#!/bin/bash
# round 4, call 1: the GPU suite + library A/B (tools/gpu_ablib.sh), the LDS-DMA fill microbenchmark, and the
# two-workgroup-per-CU GEMM configs (10, 11) against the ping-pong kernel (9) and the auto choice (0)
set -o pipefail
bash tools/gpu_ablib.sh "tests -m gpu" 2 || exit $?
timeout -k 10 300 tools/fill_bench > gpurun_out/fill_bench.txt 2>&1 || { cat gpurun_out/fill_bench.txt; exit 1; }
cat gpurun_out/fill_bench.txt
timeout -k 10 400 python -u tools/gemm_bench.py --tiles 0,9,10,11 --rounds 3 \
  --shapes fc1:8,fc2:4,qkvk:2,outk:4,fc2dgk:9,fc1dgk:1,qkvdg:1 > gpurun_out/gemm_cfg10.txt 2>&1; rc=$?
cat gpurun_out/gemm_cfg10.txt; exit $rc
