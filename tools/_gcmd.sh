for sh in sq8k sq4k fc1k4; do for t in 3 5 6; do VIT_GEMM_GROUP_M=8 timeout -k 10 60 python tools/gemm_one.py $sh $t 1 || exit 1; done; done
VIT_GEMM_GROUP_M=8 bash tools/gemm_pmc.sh sq8k 5 1
