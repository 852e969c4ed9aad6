#!/bin/bash
# SQ counter passes over one GEMM (tools/gemm_one.py args). Separate rocprofv3 runs per counter set.
set -e
export TMPDIR=/tmp
O=gpurun_out/gpmc/$1_$2_$3
mkdir -p $O
timeout -k 10 120 python3 tools/gemm_one.py "$@" > $O/plain.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex gemm_ --output-format csv -d $O/p1 -o run -- python3 tools/gemm_one.py "$@" 5 > $O/p1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_COUNT --kernel-include-regex gemm_ --output-format csv -d $O/p2 -o run -- python3 tools/gemm_one.py "$@" 5 > $O/p2.log 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gemm_ --output-format csv -d $O/p3 -o run -- python3 tools/gemm_one.py "$@" 5 > $O/p3.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex gemm_ --output-format csv -d $O/p4 -o run -- python3 tools/gemm_one.py "$@" 5 > $O/p4.log 2>&1
cat $O/plain.log
