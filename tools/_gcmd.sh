set -e
timeout -k 10 400 python -u tools/gemm_bench.py --tiles 3,5,9 --shapes fc2dgk:9/5,fc1:8/3 --rounds 3 > gpurun_out/gemm_epi89.log 2>&1
cat gpurun_out/gemm_epi89.log
