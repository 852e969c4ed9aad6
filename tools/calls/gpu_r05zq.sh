#!/bin/bash
# round 5, call 45: kernel stats of the batched column sums, abase (16 row lanes) vs the tree (64 row lanes), and a
# third B/16 A/B pair
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zq; mkdir -p $O
for t in abase .; do
  n=$(basename $t)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$n -o run -- python3 $t/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/kt_$n.log 2>&1 || { tail -5 $O/kt_$n.log; exit 1; }
  S=$(find $O/kt_$n -name "*kernel_stats.csv" | head -1)
  echo "$t:"; grep -E "colsum_batch|sgd_dev" $S | cut -d, -f1-5
  cp $S $O/stats_$n.csv; rm -rf $O/kt_$n
done
for t in abase .; do
  timeout -k 10 300 python3 -u $t/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b16_$(basename $t).json 2> $O/b16_$(basename $t).err || { tail -5 $O/b16_$(basename $t).err; exit 1; }
  echo "b16 $t: $(grep -o '"value": [0-9.]*' $O/b16_$(basename $t).json | head -1)"
done
