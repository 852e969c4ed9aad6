#!/bin/bash
# round 4, call 17: SGD stream unrolled by two (six loads in flight before the first store): standalone A/B
# against HEAD's kernel (vitmi/ab), same box
set -o pipefail
export TMPDIR=/tmp
for r in 1 2; do
  echo "base:"; VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/ab/libvit_hip.so timeout -k 10 120 python -u tools/sgd_bench.py 2>&1 | grep "n " || exit 1
  echo "new:"; timeout -k 10 120 python -u tools/sgd_bench.py 2>&1 | grep "n " || exit 1
done
