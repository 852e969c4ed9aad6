set -e
timeout -k 10 400 python -u tools/gemm_bench.py --tiles 0,9 --shapes fc1dgk:1,outk:1,qkvdg:1,fc2:4,fc1:8 --rounds 3 > gpurun_out/gemm_split.log 2>&1
cat gpurun_out/gemm_split.log
