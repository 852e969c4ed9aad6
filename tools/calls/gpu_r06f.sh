#!/bin/bash
# round 6, call 6: (1) per-step loss of the bench loop under the reference init vs the tamed init; (2) Res-ViT DP test
# incl. the graphed DP step; (3) Res-ViT-B/16 bs 128 eager vs graphed, same box (verdict item 6); (4) the N = 2
# rehearsal on one card over gloo: B/16 exchange accounting, graphed Res-ViT DP
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06f; mkdir -p $O
step() { echo "== $1"; shift; "$@" || { echo "FAILED: $*"; exit 1; }; }
step "loss trace" timeout -k 10 300 python3 -u tools/dbg/bench_loss_trace.py > $O/loss_trace.txt 2>&1
cat $O/loss_trace.txt | grep -v amdgpu.ids
step "resvit dp test" timeout -k 10 400 python -u -m pytest tests/test_resvit_train_gpu.py -x -q -k "data_parallel or share_teacher or graphed" --timeout 300 --timeout-method thread > $O/dp_test.log 2>&1
tail -2 $O/dp_test.log
for mode in graph eager graph eager; do
  if [ $mode = eager ]; then E=1; else E=0; fi
  VITMI_RESVIT_EAGER=$E step "resvit $mode" timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 20 --warmup 5 > $O/resvit_$mode.json 2> $O/resvit_$mode.err
  tail -1 $O/resvit_$mode.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('$mode', d['value'], d['ms_per_step'], d['active_ratio'])" | tee -a $O/resvit_eager_vs_graph.txt
done
VITMI_SHARE_GPU=1 VITMI_DIST_BACKEND=gloo step "b16 n2" timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 2 --steps 3 --warmup 1 --batch 32 > $O/b16_n2.json 2> $O/b16_n2.err
tail -1 $O/b16_n2.json | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['value'],d['n_gpus'],d['config']['dist_backend'],json.dumps(d.get('dist_check')))"
VITMI_SHARE_GPU=1 VITMI_DIST_BACKEND=gloo step "resvit n2" timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29572 bench.py --arch resvit_b16 --gpus 2 --steps 3 --warmup 1 --batch 16 > $O/resvit_n2.json 2> $O/resvit_n2.err
tail -1 $O/resvit_n2.json | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['value'],d['n_gpus'],d['config']['workload'],json.dumps(d.get('dist_check')))"
