set -e
timeout -k 10 300 python -u tools/gemm_bench.py --tiles 3,5,9 --shapes out:1,fc1:1 --rounds 2 > gpurun_out/gemm_outdg.log 2>&1
cat gpurun_out/gemm_outdg.log
bash tools/gpu_check.sh tests bench
