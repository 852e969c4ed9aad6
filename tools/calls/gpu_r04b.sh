#!/bin/bash
# round 4, call 2: LDS-DMA / VGPR-load / store rates per CU (tools/fill_bench), the counter list, and the L2
# hit rate of the fc1 forward GEMM's main loop
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04b
timeout -k 10 300 tools/fill_bench > gpurun_out/r04b/fill_bench.txt 2>&1 || { cat gpurun_out/r04b/fill_bench.txt; exit 1; }
cat gpurun_out/r04b/fill_bench.txt
timeout -k 10 60 rocprofv3 -L > gpurun_out/r04b/counters.txt 2>&1 || true
grep -o "\b\(TA\|TD\|TCP\|TCC\)_[A-Z_a-z0-9]*" gpurun_out/r04b/counters.txt | sort -u | tr '\n' ' ' | head -c 6000; echo
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex gemm_ --output-format csv -d gpurun_out/r04b/tcc -o run -- python3 tools/gemm_one.py fc1 9 1 5 > gpurun_out/r04b/tcc.log 2>&1 || { tail -5 gpurun_out/r04b/tcc.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r04b/tcc/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    agg[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(k, sum(v) / len(v))
PY
