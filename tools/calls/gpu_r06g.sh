#!/bin/bash
# round 6, call 7: the bench with the conditioned init (finite losses) vs the raw reference init (NaN from step 1), same
# box, two rounds each; the Res-ViT bench's losses
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06g; mkdir -p $O
step() { echo "== $1"; shift; "$@" || { echo "FAILED: $*"; exit 1; }; }
for r in 1 2; do
  for init in conditioned reference; do
    VITMI_BENCH_INIT=$init step "b16 $init $r" timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b16_${init}_$r.json 2> $O/b16_${init}_$r.err
    tail -1 $O/b16_${init}_$r.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('$init', d['value'], d['ms_per_step'], d['loss_first_timed_step'], d['loss_last_timed_step'], d.get('train_epoch_img_s'), d['roofline']['frac'], d['roofline_fwd_dgrad']['frac'])" | tee -a $O/init_ab.txt
  done
done
step "resvit" timeout -k 10 300 python3 -u bench.py --arch resvit_b16 --steps 20 --warmup 5 > $O/resvit.json 2> $O/resvit.err
tail -1 $O/resvit.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['loss_first_timed_step'], d['loss_last_timed_step'])"
