#!/bin/bash
# round 6, call 4: w4 prototype, LDS-DMA variant (w4d) vs register staging, ablations
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06d; mkdir -p $O
step() { echo "== $1"; shift; "$@" || { echo "FAILED: $*"; exit 1; }; }
for sh in "50432 768 3072" "50432 768 2304" "50432 768 768" "50432 3072 768"; do
  W4_DIAG=1 step "proto $sh" timeout -k 10 120 tools/w4_proto $sh >> $O/proto.txt 2>&1
done
cat $O/proto.txt
step "new tests" timeout -k 10 600 python -u -m pytest tests/test_optim_dev_gpu.py tests/test_resvit_gpu.py tests/test_resvit_train_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
step "bench b16" timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_b16.json 2> $O/bench_b16.err
python3 -c "import json; d=json.load(open('$O/bench_b16.json')); print(d['value'], d['ms_per_step'], d.get('train_epoch_img_s'), d.get('train_epoch_vs_value'), d['roofline']['frac'], d['roofline_fwd_dgrad']['frac'])"
