#!/bin/bash
# round 4, call 14: persistent attention forward (attention_fwd_pers.hip): attention tests, standalone A/B
# against the one-shot kernel (path 3) at B/16 bs 256, L/16 bs 64, tiny / many-item shapes, then B/16 bs 256
# bench with the persistent forward vs the one-shot path (VITMI_ATTN_PATH=3), same box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 100 python -u tools/dbg_attn_fwd_pers.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/attn_bench.py 256 197 12 64 0 256 197 12 64 3 64 197 16 64 0 64 197 16 64 3 256 197 12 64 0 256 197 12 64 3 2>&1 | grep -v amdgpu.ids | grep fwd || exit 1
for r in 1 2; do
  for pth in 0 3; do
    VITMI_ATTN_FWD_PATH=$pth timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b16_p${pth}_$r.json 2> $O/b16_p${pth}_$r.err || { tail -5 $O/b16_p${pth}_$r.err; exit 1; }
    echo "attn fwd path=$pth run $r: $(grep -o '"value": [0-9.]*' $O/b16_p${pth}_$r.json | head -1)"
  done
done
