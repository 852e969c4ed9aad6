#!/bin/bash
# round 5, call 35: speed only of the delta-from-O attention backward (its parity failed the 3e-2 gradient bar on the
# query weights in test_b16_full_gradients_match_oracle): standalone bwd times and a same-box B/16 A/B against abase
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zg; mkdir -p $O
for t in abase .; do
  timeout -k 10 120 python3 -u $t/tools/attn_bench.py 256 197 12 64 0 128 197 12 64 0 64 197 16 64 0 > $O/attn_$(basename $t).txt 2>&1 || { tail -5 $O/attn_$(basename $t).txt; exit 1; }
  echo "$t:"; grep bwd $O/attn_$(basename $t).txt
done
for t in abase .; do
  timeout -k 10 300 python3 -u $t/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b16_$(basename $t).json 2> $O/b16_$(basename $t).err || { tail -5 $O/b16_$(basename $t).err; exit 1; }
  echo "$t: $(grep -o '"value": [0-9.]*' $O/b16_$(basename $t).json | head -1)"
done
