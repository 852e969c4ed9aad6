#!/bin/bash
# round 5, call 26: batched padded casts (vit_cast_pad_batch: the LoRA pack, the router / approximator weight pads,
# the backward's B_z casts, one launch each): tests, then same-box Res-ViT A/B against d5859ad (abase)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05y; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_resvit_gpu.py tests/test_resvit_train_gpu.py -x -q \
  --timeout 300 --timeout-method thread -k "cast or splitk or segment_colsum or resvit or router or approx or graphed or fused or trajectory or reference or lora" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  (cd abase && timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 10 --warmup 3 --no-cpu-baseline > ../$O/base_$r.json 2> ../$O/base_$r.err) || { tail -5 $O/base_$r.err; exit 1; }
  timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 10 --warmup 3 --no-cpu-baseline > $O/new_$r.json 2> $O/new_$r.err || { tail -5 $O/new_$r.err; exit 1; }
  echo "run $r base: $(grep -o '"value": [0-9.]*' $O/base_$r.json | head -1)  new: $(grep -o '"value": [0-9.]*' $O/new_$r.json | head -1)"
done
