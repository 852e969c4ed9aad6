#!/bin/bash
# round 6, call 16: LDS counters of gemm_pp2 (K-contiguous forward vs the M/N-contiguous split-K weight gradient):
# bank-conflict cycles against all LDS-array cycles, LDS instructions
set -o pipefail
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r06p; mkdir -p $O
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
timeout -k 10 -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "gemm_pp2" --output-format csv -d $O/pmc -o run -- python3 $R/tools/gemm_bench.py --tiles 0 --rounds 1 --shapes fc2:4,qkvdg:1,fc1dg:1 --wgrad --splits 7 > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
f=$(find $O/pmc -name "*counter_collection.csv" | head -1)
cp $f $O/lds_pmc.csv
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float); n = collections.Counter()
for r in rows:
    k = (r["Kernel_Name"][:80], r["Counter_Name"])
    agg[k] += float(r["Counter_Value"]); n[k] += 1
for k, v in sorted(agg.items()):
    print(f"{k[0]:80s} {k[1]:22s} {v / n[k]:16.0f}  (x{n[k]})")
PY
