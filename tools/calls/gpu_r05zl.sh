#!/bin/bash
# round 5, call 40: the SGD step with non-temporal loads / stores: tools/sgd_bench.py and B/16 A/B against abase (HEAD)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zl; mkdir -p $O
for t in abase .; do
  timeout -k 10 120 python3 -u $t/tools/sgd_bench.py > $O/sgd_$(basename $t).txt 2>&1 || { tail -5 $O/sgd_$(basename $t).txt; exit 1; }
  echo "$t:"; cat $O/sgd_$(basename $t).txt | grep "n "
done
for r in 1 2; do
  for t in abase .; do
    timeout -k 10 300 python3 -u $t/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b16_$(basename $t)_$r.json 2> $O/b16_$(basename $t)_$r.err || { tail -5 $O/b16_$(basename $t)_$r.err; exit 1; }
    echo "$t run $r: $(grep -o '"value": [0-9.]*' $O/b16_$(basename $t)_$r.json | head -1)"
  done
done
