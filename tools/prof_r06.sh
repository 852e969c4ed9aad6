#!/bin/bash
# Round-6 evidence for profiles/r06/: the full GPU test suite, smoke(), the default bench line (with
# the CPU baseline), its kernel trace + step timeline, and separate --pmc passes (FETCH_SIZE; WRITE_SIZE; MFMA
# busy) for the roofline kernels (split-K weight gradient, fc1 forward) and the attention backward.
# usage: bash tools/prof_r06.sh TAG [skip-tests|tests] [graph]
set -o pipefail
export TMPDIR=/tmp
# the profiled runs skip the train_epoch leg (its steps would shift the per-step trace windows)
export VITMI_BENCH_TRAIN_EPOCH=0
TAG=${1:-v1}
O=gpurun_out/r06_prof_$TAG
mkdir -p $O
step() { echo "== $1"; shift; "$@" || { echo "FAILED: $*"; exit 1; }; }
if [ "$2" != "skip-tests" ]; then
  step "pytest -m gpu" timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  tail -2 $O/gpu_tests.log
  step "smoke" timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
  tail -1 $O/smoke.log
fi
step "bench" env VITMI_BENCH_TRAIN_EPOCH=1 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_b16.json 2> $O/bench_b16.err
tail -c 400 $O/bench_b16.json; echo
step "ktrace" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/ktrace.log 2>&1
S=$(find $O/ktrace -name "*kernel_stats.csv" | head -1)
T=$(find $O/ktrace -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py $S 13 > $O/kernel_summary.txt
python3 tools/trace_step.py $T 3 $O/step_launches.txt > $O/step_timeline.txt
cp $S $O/kernel_stats.csv
rm -rf $O/ktrace
RX='gemm_pp2_kernel<false, false, 7|gemm_pp2_group_kernel|gemm_\w+_kernel<.*true, true, 8|attn_bwd_pers_kernel'
step "pmc fetch" timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/fetch.log 2>&1
step "pmc write" timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/write.log 2>&1
step "pmc mfma" timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-include-regex "$RX" --output-format csv -d $O/mfma -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/mfma.log 2>&1
F=$(find $O/fetch -name "*counter_collection.csv" | head -1)
W=$(find $O/write -name "*counter_collection.csv" | head -1)
M=$(find $O/mfma -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py 'gemm_pp2_kernel<false, false, 7' $F $W $O/wgrad_traffic.json > /dev/null
python3 tools/pmc_traffic.py 'gemm_\w+_kernel<.*true, true, 8' $F $W $O/fc1_traffic.json > /dev/null
python3 tools/pmc_traffic.py 'attn_bwd_pers_kernel' $F $W $O/attn_bwd_traffic.json > /dev/null
python3 tools/pmc_traffic.py 'gemm_pp2_group_kernel' $F $W $O/wgrad_group_traffic.json > /dev/null
python3 tools/kernel_pmc.py $O/kernel_pmc.txt $F $W $M
cp $F $O/fetch.csv; cp $W $O/write.csv; cp $M $O/mfma.csv
rm -rf $O/fetch $O/write $O/mfma
head -30 $O/kernel_summary.txt; head -4 $O/step_timeline.txt
python3 -c "import json;[print(k, round(json.load(open('$O/'+k))['traffic_bytes']/1e6,1),'MB') for k in ['wgrad_traffic.json','wgrad_group_traffic.json','fc1_traffic.json','attn_bwd_traffic.json']]"
head -30 $O/kernel_pmc.txt
# same-box A/B: the whole B/16 step replayed from one HIP graph (VITMI_BENCH_GRAPH=1) vs eager launches
[ "$3" == "graph" ] || exit 0
for r in 1 2; do
  for gr in 0 1; do
    VITMI_BENCH_GRAPH=$gr timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b16_graph${gr}_$r.json 2> $O/b16_graph${gr}_$r.err || { tail -5 $O/b16_graph${gr}_$r.err; exit 1; }
    echo "graph=$gr run $r: $(grep -o '"value": [0-9.]*' $O/b16_graph${gr}_$r.json | head -1)"
  done
done
