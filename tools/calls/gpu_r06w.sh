#!/bin/bash
# round 6, call 23: the N>1 bench path on the final tree, rehearsed as 2 gloo ranks sharing the one GPU (replica check,
# exchange accounting); B/16 and Res-ViT
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06w; mkdir -p $O
step() { echo "== $1"; shift; "$@" || { echo "FAILED: $*"; exit 1; }; }
VITMI_SHARE_GPU=1 VITMI_DIST_BACKEND=gloo step "b16 n2" timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 2 --steps 3 --warmup 1 --batch 32 > $O/b16_n2.json 2> $O/b16_n2.err
tail -1 $O/b16_n2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['dist_check']['replicas_identical'], d['dist_check']['exchange'])"
VITMI_SHARE_GPU=1 VITMI_DIST_BACKEND=gloo step "resvit n2" timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29572 bench.py --arch resvit_b16 --gpus 2 --steps 3 --warmup 1 --batch 16 > $O/resvit_n2.json 2> $O/resvit_n2.err
tail -1 $O/resvit_n2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['dist_check']['replicas_identical'])"
