#!/bin/bash
# round 5, call 22: debug — which Res-ViT parameters' gradients differ between two gloo DP replicas with the LoRA sinks,
# and the reducer's mark count per parameter; then the DP test and the Res-ViT training tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29561 tools/dbg/resvit_dp_diff.py > $O/dp_diff.log 2>&1 || { tail -30 $O/dp_diff.log; exit 1; }
grep -v "^\[W\|amdgpu.ids\|Gloo" $O/dp_diff.log | cut -c1-300 | head -30
timeout -k 10 600 python -u -m pytest tests/test_resvit_train_gpu.py tests/test_resvit_gpu.py tests/test_train_gpu.py -q -x --timeout 250 --timeout-method thread > $O/tests.log 2>&1; echo "tests: $(tail -1 $O/tests.log)"
