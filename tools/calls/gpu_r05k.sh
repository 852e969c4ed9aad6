#!/bin/bash
# round 5, call 12: grouped out-projection + q|k|v weight gradients (vit_gemm_splitk_group): kernel tests, the
# engine parity tests that cover the backward, then same-box bench A/B (VITMI_GROUP_WGRAD=0 / 1) on B/16 and L/16
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "splitk or parts_equal or wave_split or gradients or step_matches or side_stream or pruning or large_arch" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for a in "b16" "l16 --batch 64"; do
  t=$(echo $a | cut -d' ' -f1)
  for r in 1 2; do
    for gw in 0 1; do
      VITMI_GROUP_WGRAD=$gw timeout -k 10 300 python3 -u bench.py --arch $a --steps 20 --warmup 5 --no-cpu-baseline > $O/${t}_g${gw}_$r.json 2> $O/${t}_g${gw}_$r.err || { tail -5 $O/${t}_g${gw}_$r.err; exit 1; }
      echo "$t group=$gw run $r: $(grep -o '"value": [0-9.]*' $O/${t}_g${gw}_$r.json | head -1)"
    done
  done
done
