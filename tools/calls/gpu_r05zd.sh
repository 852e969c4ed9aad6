#!/bin/bash
# round 5, call 32: host-side time of the graphed Res-ViT step (tools/dbg/resvit_host_time.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zd; mkdir -p $O
timeout -k 10 300 python3 -u tools/dbg/resvit_host_time.py > $O/host_time.txt 2>&1 || { tail -20 $O/host_time.txt; exit 1; }
tail -3 $O/host_time.txt
