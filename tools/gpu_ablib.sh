#!/bin/bash
# A/B in one call: optional pytest selection ($1, "" = none), then the default bench line with the baseline
# library (vitmi/ab/libvit_hip.so, tools/ab_tree.sh / ab_build.sh; remove ./vit-of-pytorch_amd/vitmi/ab from
# .gpurunignore for the call) and with this tree's library, alternately, $2 rounds (default 2). Extra bench
# flags in $3.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
if [ -n "$1" ]; then
  timeout -k 10 900 python -u -m pytest $1 -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for i in $(seq 1 ${2:-2}); do
  VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/ab/libvit_hip.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline $3 > $O/base_$i.json 2> $O/base_$i.err || { tail -3 $O/base_$i.err; exit 1; }
  echo "base: $(grep -o '"value": [0-9.]*' $O/base_$i.json)"
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline $3 > $O/new_$i.json 2> $O/new_$i.err || { tail -3 $O/new_$i.err; exit 1; }
  echo "new:  $(grep -o '"value": [0-9.]*' $O/new_$i.json)"
done
