set -e
timeout -k 10 400 python -u tools/gemm_bench.py --tiles 3,5 --shapes fc1:3,fc2:4,qkv:2,out:4,fc2dg:5,fc1dg:1,qkvdg:1,out:1 --rounds 2 --wgrad --splits 4,7,9,16,28 > gpurun_out/gemm_epi.log 2>&1
cat gpurun_out/gemm_epi.log
