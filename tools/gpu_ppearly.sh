#!/bin/bash
# gemm_pp_kernel DMA issue placement (VIT_GEMM_PP_EARLY = 1 / 2): stamps + timing of the split-K weight
# gradients, GEMM tests under each setting, then bench A/B (alternately)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ppe; mkdir -p $O
for e in 1 2; do
  VIT_GEMM_PP_EARLY=$e timeout -k 10 60 tools/gdiag_bin 3072 768 50432 5 7 3 1 1 7 > $O/st_$e.txt 2>&1 || exit 1
  python tools/diag_slots.py $O/st_$e.txt | head -9
  VIT_GEMM_PP_EARLY=$e timeout -k 10 60 tools/gdiag_bin 2304 768 50432 5 7 -1 1 1 9 | head -1
  VIT_GEMM_PP_EARLY=$e timeout -k 10 60 tools/gdiag_bin 768 768 50432 5 7 -1 1 1 28 | head -1
  VIT_GEMM_PP_EARLY=$e timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm or wgrad or splitk" -x -q --timeout 200 --timeout-method thread > $O/tests_$e.log 2>&1
  rc=$?; tail -1 $O/tests_$e.log; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for e in 1 2; do
    VIT_GEMM_PP_EARLY=$e timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b${e}_$i.json 2> $O/b${e}_$i.err || { tail -3 $O/b${e}_$i.err; exit 1; }
    echo "early=$e: $(grep -o '"value": [0-9.]*' $O/b${e}_$i.json) $(grep -o '"frac": [0-9.]*' $O/b${e}_$i.json | head -1)"
  done
done
