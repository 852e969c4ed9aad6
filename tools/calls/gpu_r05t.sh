#!/bin/bash
# round 5, call 21: the Res-ViT DP test with and without the LoRA gradient sinks; with sinks and serialized launches;
# the single-process Res-ViT training tests with sinks
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05t; mkdir -p $O
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u -m pytest tests/test_resvit_train_gpu.py -x -q --timeout 250 --timeout-method thread -k "data_parallel" > $O/dp_sink_serial.log 2>&1; echo "sink, serialized kernels: $(tail -1 $O/dp_sink_serial.log)"
timeout -k 10 600 python -u -m pytest tests/test_resvit_train_gpu.py tests/test_resvit_gpu.py -q --timeout 250 --timeout-method thread -k "not data_parallel" > $O/sp_sink.log 2>&1; echo "single-process, sink: $(tail -1 $O/sp_sink.log)"
grep -E "^FAILED" $O/sp_sink.log | head
