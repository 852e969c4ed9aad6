#!/bin/bash
# A/B of one architecture's bench line: ./abase (tools/ab_tree.sh) vs this tree, alternately, in one call.
#   bash tools/gpu_arch_ab.sh <arch> [rounds] [steps]
set -o pipefail
export TMPDIR=/tmp
A=${1:-h14}; O=gpurun_out/ab_$A; mkdir -p $O
for i in $(seq 1 ${2:-2}); do
  timeout -k 10 300 python -u abase/bench.py --arch $A --steps ${3:-10} --warmup 3 --no-cpu-baseline > $O/base_$i.json 2> $O/base_$i.err || { tail -3 $O/base_$i.err; exit 1; }
  echo "base: $(grep -o '"value": [0-9.]*' $O/base_$i.json)"
  timeout -k 10 300 python -u bench.py --arch $A --steps ${3:-10} --warmup 3 --no-cpu-baseline > $O/new_$i.json 2> $O/new_$i.err || { tail -3 $O/new_$i.err; exit 1; }
  echo "new:  $(grep -o '"value": [0-9.]*' $O/new_$i.json)"
done
