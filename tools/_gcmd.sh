set -e
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/gemm_bench.py --tiles 9 --shapes fc1:8/1 --rounds 3
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_dropout_gpu.py tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1; tail -1 gpurun_out/bench.log | cut -c1-200; tail -1 gpurun_out/bench.log | grep -o '"roofline.*"step_mfma_frac": [0-9.]*'
