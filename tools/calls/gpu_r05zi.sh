#!/bin/bash
# round 5, call 37: the routed block input passed through the fused router node (its LN backward adds the layer input gradient): Res-ViT tests, then same-box
# A/B VITMI_RESVIT_NO_ROUTER_THROUGH=1/0
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zi; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_resvit_gpu.py tests/test_resvit_train_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    VITMI_RESVIT_NO_ROUTER_THROUGH=$v timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 10 --warmup 3 --no-cpu-baseline > $O/nt${v}_$r.json 2> $O/nt${v}_$r.err || { tail -5 $O/nt${v}_$r.err; exit 1; }
    echo "no_router_through=$v run $r: $(grep -o '"value": [0-9.]*' $O/nt${v}_$r.json | head -1)"
  done
done
