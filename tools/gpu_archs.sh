#!/bin/bash
# one bench line per other configuration (L/16, H/14, Res-ViT-B/16) for profiles/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/archs; mkdir -p $O
for a in l16 h14 resvit_b16; do
  timeout -k 10 300 python -u bench.py --arch $a --steps 10 --warmup 3 --no-cpu-baseline > $O/$a.json 2> $O/$a.err || { tail -3 $O/$a.err; exit 1; }
  echo "$a: $(grep -o '"value": [0-9.]*' $O/$a.json) $(grep -o '"frac": [0-9.]*' $O/$a.json | head -1)"
done
