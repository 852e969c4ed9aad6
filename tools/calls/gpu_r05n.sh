#!/bin/bash
# round 5, call 15: where the Res-ViT-B/16 step's remaining glue comes from (torch.profiler, tools/resvit_prof.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 400 python3 -u tools/resvit_prof.py > $O/resvit_prof.txt 2>&1 || { tail -20 $O/resvit_prof.txt; exit 1; }
tail -120 $O/resvit_prof.txt
