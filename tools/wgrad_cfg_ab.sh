export TMPDIR=/tmp
timeout -k 10 120 python -u tools/gemm_bench.py --tiles 5,9 --shapes "" --wgrad --splits 7,9,28 --rounds 1
bash tools/bench_env.sh VIT_GEMM_SPLITK_CFG=5 VIT_GEMM_SPLITK_CFG=9
