#!/bin/bash
# SQ counter passes over the attention kernels of tools/attn_bench.py (default ViT-B/16 bs256 shape);
# one rocprofv3 run per counter set (gfx950 limits: <= 8 SQ counters per pass). $1 = tree (default .)
set -o pipefail
export TMPDIR=/tmp
T=${1:-.}
O=gpurun_out/apmc_$(basename $(realpath $T))
rm -rf $O; mkdir -p $O
timeout -k 10 120 python3 $T/tools/attn_bench.py > $O/plain.log 2>&1 || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex attn_ --output-format csv -d $O/p1 -o run -- python3 $T/tools/attn_bench.py > $O/p1.log 2>&1 || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU GRBM_COUNT --kernel-include-regex attn_ --output-format csv -d $O/p2 -o run -- python3 $T/tools/attn_bench.py > $O/p2.log 2>&1 || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_VMEM GRBM_COUNT --kernel-include-regex attn_ --output-format csv -d $O/p3 -o run -- python3 $T/tools/attn_bench.py > $O/p3.log 2>&1 || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM GRBM_COUNT --kernel-include-regex attn_ --output-format csv -d $O/p4 -o run -- python3 $T/tools/attn_bench.py > $O/p4.log 2>&1 || exit 1
python3 - "$O" <<'PY'
import csv, glob, collections, sys
O = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{O}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(f"{O}/summary.txt", "w") as out:
    for k, cs in agg.items():
        out.write(k + "\n")
        for c, v in sorted(cs.items()):
            out.write(f"   {c:28s} {sum(v)/len(v):16.1f}  (n={len(v)})\n")
print(open(f"{O}/summary.txt").read())
PY
cat $O/plain.log
