#!/bin/bash
# round 5, call 24: branch-free router gate kernel (loads of 8 rows in flight), the router output-bias sum folded into
# the batched column sums: tests, Res-ViT A/B against a24080b (abase), the gate under torch.profiler
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_resvit_gpu.py tests/test_resvit_train_gpu.py -x -q \
  --timeout 300 --timeout-method thread -k "splitk or segment_colsum or resvit or router or approx or graphed or fused or trajectory or reference or lora or sink" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  (cd abase && timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 10 --warmup 3 --no-cpu-baseline > ../$O/base_$r.json 2> ../$O/base_$r.err) || { tail -5 $O/base_$r.err; exit 1; }
  timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 10 --warmup 3 --no-cpu-baseline > $O/new_$r.json 2> $O/new_$r.err || { tail -5 $O/new_$r.err; exit 1; }
  echo "run $r base: $(grep -o '"value": [0-9.]*' $O/base_$r.json | head -1)  new: $(grep -o '"value": [0-9.]*' $O/new_$r.json | head -1)"
done
timeout -k 10 400 python3 -u tools/resvit_prof.py > $O/resvit_prof.txt 2>&1 || { tail -20 $O/resvit_prof.txt; exit 1; }
grep -E "router_dx_gate|segment_colsum|colsum_partial|Self CUDA" $O/resvit_prof.txt | head -5
