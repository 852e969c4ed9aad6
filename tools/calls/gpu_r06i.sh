#!/bin/bash
# round 6, call 9: evidence v2 on the current tree — full -m gpu suite, smoke(), the default bench line (CPU baseline
# included), the DP configs' per-rank shapes and Res-ViT on finite numbers
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06i; mkdir -p $O
step() { echo "== $1"; shift; "$@" || { echo "FAILED: $*"; exit 1; }; }
step "pytest -m gpu" timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log
step "smoke" timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
step "bench b16" timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_b16.json 2> $O/bench_b16.err
tail -1 $O/bench_b16.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('b16', d['value'], d['ms_per_step'], d['loss_first_timed_step'], d['loss_last_timed_step'], d.get('train_epoch_img_s'), d['roofline']['frac'], d['roofline_fwd_dgrad']['frac'], d['step_mfma_frac_algorithmic'], d['cpu_baseline']['value'])"
for a in "l16 64" "h14 128"; do set -- $a
  step "bench $1" timeout -k 10 400 python3 -u bench.py --arch $1 --batch $2 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$1_bs$2.json 2> $O/bench_$1.err
  tail -1 $O/bench_$1_bs$2.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('$1', d['value'], d['ms_per_step'], d['loss_first_timed_step'], d['loss_last_timed_step'], d['step_mfma_frac_algorithmic'])"
done
step "bench resvit" timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 20 --warmup 5 > $O/bench_resvit_b16.json 2> $O/bench_resvit.err
tail -1 $O/bench_resvit_b16.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('resvit', d['value'], d['ms_per_step'], d['loss_first_timed_step'], d['loss_last_timed_step'])"
