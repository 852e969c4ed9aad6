set -e
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/ln_bench.py
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_dropout_gpu.py -k "layernorm" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
