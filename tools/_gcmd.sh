set -e
timeout -k 10 400 python -u tools/gemm_bench.py --tiles 3,5,9 --shapes qkvk:2,outk:4,fc2dgk:5,fc1dgk:1,outk:1 --rounds 2 > gpurun_out/gemm_kc.log 2>&1
cat gpurun_out/gemm_kc.log
bash tools/gpu_check.sh tests bench
