#!/bin/bash
# stage-1 stamps of the attention backward, then the round-3 evidence set (tools/prof_r03.sh)
set -o pipefail
export TMPDIR=/tmp
VITMI_LIB=$PWD/vit-of-pytorch_amd/vitmi/ab/libvit_hip.so timeout -k 10 120 python tools/attn_stamps.py 2>&1 | grep wave || exit 1
bash tools/prof_r03.sh ${1:-v2}
