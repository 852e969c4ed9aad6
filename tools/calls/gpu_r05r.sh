#!/bin/bash
# round 5, call 19: grouped split-K reductions (vit_splitk_reduce_group) in the engine's grouped weight gradients, the
# router / approximator gradients and the fused layer's LoRA gradients (dB | dA one grouped launch): tests, then
# same-box bench A/B against a24080b (abase) on Res-ViT-B/16 and B/16
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py tests/test_resvit_gpu.py tests/test_resvit_train_gpu.py -x -q \
  --timeout 300 --timeout-method thread -k "splitk or segment_colsum or resvit or router or approx or graphed or fused or trajectory or reference or gradients or step_matches or pruning" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for a in resvit_b16 b16; do
  for r in 1 2; do
    (cd abase && timeout -k 10 300 python3 -u bench.py --arch $a --steps 10 --warmup 3 --no-cpu-baseline > ../$O/base_${a}_$r.json 2> ../$O/base_${a}_$r.err) || { tail -5 $O/base_${a}_$r.err; exit 1; }
    timeout -k 10 300 python3 -u bench.py --arch $a --steps 10 --warmup 3 --no-cpu-baseline > $O/new_${a}_$r.json 2> $O/new_${a}_$r.err || { tail -5 $O/new_${a}_$r.err; exit 1; }
    echo "$a run $r base: $(grep -o '"value": [0-9.]*' $O/base_${a}_$r.json | head -1)  new: $(grep -o '"value": [0-9.]*' $O/new_${a}_$r.json | head -1)"
  done
done
