#!/bin/bash
# round 6, call 10: the forward attention's key-split last strip (verdict item 3): kernel tests, the bs-256 gradient
# test, attn_bench and the B/16 bench line, new vs HEAD's kernel (vitmi/ab), same box, interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06j; mkdir -p $O
step() { echo "== $1"; shift; "$@" || { echo "FAILED: $*"; exit 1; }; }
step "attn tests" timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
step "parity tests" timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1
tail -2 $O/parity.log
AB=$PWD/vit-of-pytorch_amd/vitmi/ab/libvit_hip.so
for r in 1 2 3; do
  step "attn new $r" timeout -k 10 120 python3 -u tools/attn_bench.py 256 197 12 64 0 64 197 16 64 0 >> $O/attn_new.txt 2>&1
  VITMI_LIB=$AB step "attn old $r" timeout -k 10 120 python3 -u tools/attn_bench.py 256 197 12 64 0 64 197 16 64 0 >> $O/attn_old.txt 2>&1
done
echo new; grep fwd $O/attn_new.txt; echo old; grep fwd $O/attn_old.txt
for r in 1 2; do
  step "bench new $r" timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_new_$r.json 2> $O/b_new_$r.err
  VITMI_LIB=$AB step "bench old $r" timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_old_$r.json 2> $O/b_old_$r.err
  for v in new old; do tail -1 $O/b_${v}_$r.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('$v', d['value'], d['ms_per_step'], d['loss_last_timed_step'])" | tee -a $O/bench_ab.txt; done
done
