#!/bin/bash
# round 5, call 34: attention backward stage 1 with delta = rowsum(dO * O) and streamed key-tile pairs: attention
# tests and the training-parity tests, then standalone bwd times (tools/attn_bench.py) and same-box B/16 A/B against
# abase (HEAD before the change)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05zf; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 300 --timeout-method thread > $O/tests_attn.log 2>&1 || { tail -60 $O/tests_attn.log; exit 1; }
tail -1 $O/tests_attn.log
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_train_gpu.py tests/test_resvit_gpu.py tests/test_submodules_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests_parity.log 2>&1 || { tail -60 $O/tests_parity.log; exit 1; }
tail -1 $O/tests_parity.log
for t in abase .; do
  timeout -k 10 120 python3 -u $t/tools/attn_bench.py 256 197 12 64 0 128 197 12 64 0 64 197 16 64 0 > $O/attn_$(basename $t).txt 2>&1 || { tail -5 $O/attn_$(basename $t).txt; exit 1; }
  echo "$t:"; grep bwd $O/attn_$(basename $t).txt
done
for r in 1 2; do
  for t in abase .; do
    timeout -k 10 300 python3 -u $t/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b16_$(basename $t)_$r.json 2> $O/b16_$(basename $t)_$r.err || { tail -5 $O/b16_$(basename $t)_$r.err; exit 1; }
    echo "$t run $r: $(grep -o '"value": [0-9.]*' $O/b16_$(basename $t)_$r.json | head -1)"
  done
done
