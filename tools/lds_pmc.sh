#!/bin/bash
# LDS bank-conflict / activity counters of the ping-pong GEMMs (tools/gemm_diag build): the split-K fc1
# weight gradient (M/N-contiguous operands, transpose reads) and the fc2 forward (K-contiguous, b128 reads)
set -o pipefail
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/ldsp; mkdir -p $O
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16"
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "gemm_pp" --output-format csv -d $O/wg -o run -- $R/tools/gdiag_bin 3072 768 50432 5 7 -1 1 1 7 > $O/wg.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "gemm_pp" --output-format csv -d $O/fc2 -o run -- $R/tools/gdiag_bin 50432 768 3072 9 4 -1 0 0 1 > $O/fc2.log 2>&1 || exit 1
cd $R
for d in wg fc2; do
  f=$(find $O/$d -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float); n = collections.Counter()
for r in rows:
    k = (r["Kernel_Name"][:70], r["Counter_Name"])
    agg[k] += float(r["Counter_Value"]); n[k] += 1
for k, v in sorted(agg.items()):
    print(k[0], k[1], round(v / n[k]))
PY
done
