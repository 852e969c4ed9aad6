#!/bin/bash
# round 5, call 46: the N = 2 rehearsal (two ranks on one card over gloo) repeated on the final tree (Res-ViT router pass-through, fused embedding, routing masks)
# replica hash check, per-rank timing, the gradient bucket exchange) for B/16 at a small batch, and Res-ViT
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zr; mkdir -p $O
VITMI_SHARE_GPU=1 VITMI_DIST_BACKEND=gloo timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 2 --steps 3 --warmup 1 --batch 32 > $O/b16_n2.json 2> $O/b16_n2.err || { tail -20 $O/b16_n2.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/b16_n2.json').read().strip().splitlines()[-1]);print(d['value'],d['n_gpus'],d['config']['dist_backend'],json.dumps(d.get('dist_check'))[:400])"
VITMI_SHARE_GPU=1 VITMI_DIST_BACKEND=gloo timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29572 bench.py --arch resvit_b16 --gpus 2 --steps 3 --warmup 1 --batch 16 > $O/resvit_n2.json 2> $O/resvit_n2.err || { tail -20 $O/resvit_n2.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/resvit_n2.json').read().strip().splitlines()[-1]);print(d['value'],d['n_gpus'],json.dumps(d.get('dist_check'))[:400])"
