#!/bin/bash
# SQ counter passes over the attention kernels (tools/attn_bench.py, ViT-B/16 bs256), separate rocprofv3 runs
# per counter set; VARIANTS = values of VIT_ATTN_FWD_VARIANT to profile (default: 0).
set -e
export TMPDIR=/tmp
for V in ${VARIANTS:-0}; do
O=gpurun_out/apmc_v$V
mkdir -p $O
export VIT_ATTN_FWD_VARIANT=$V
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex attn_ --output-format csv -d $O/p1 -o run -- python3 tools/attn_bench.py > $O/p1.log 2>&1
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU GRBM_COUNT --kernel-include-regex attn_ --output-format csv -d $O/p2 -o run -- python3 tools/attn_bench.py > $O/p2.log 2>&1
timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex attn_ --output-format csv -d $O/p3 -o run -- python3 tools/attn_bench.py > $O/p3.log 2>&1
timeout -k 10 -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex attn_ --output-format csv -d $O/p4 -o run -- python3 tools/attn_bench.py > $O/p4.log 2>&1
for k in ${KERNELS:-attn_fwd attn_bwd}; do echo "== variant $V $k"; python3 tools/pmc_table.py $(find $O/p1 $O/p2 $O/p3 $O/p4 -name "*counter_collection.csv") --kernel ${k}; done
done
