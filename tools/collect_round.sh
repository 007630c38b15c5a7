#!/bin/bash
# Copy the judged outputs of `TAG=<tag> tools/round.sh` from gpurun_out/ into profiles/ (<tag>_* files, the
# counter jsons the bench line reads).  Run here, after the gpurun call has merged gpurun_out/ back.
set -e
cd "$(dirname "$0")/.."
T=${1:?tag}; O=gpurun_out; P=profiles
cp $O/bench_$T.json $P/${T}_bench.json
cp $O/prof_bench_$T.json $P/${T}_prof_bench.json
cp $O/prof_$T/run_kernel_stats.csv $P/${T}_kernel_stats.csv
cp $O/trace_busy_$T.json $P/${T}_trace_busy.json
[ -f $O/pytest_gpu_$T.log ] && cp $O/pytest_gpu_$T.log $P/${T}_pytest_gpu.log
[ -f $O/smoke_$T.log ] && cp $O/smoke_$T.log $P/${T}_smoke.log
mkdir -p $P/${T}_pmc $P/${T}_sq
cp $O/pmc_${T}_FETCH_SIZE/run_counter_collection.csv $P/${T}_pmc/fetch_size_counter_collection.csv
cp $O/pmc_${T}_WRITE_SIZE/run_counter_collection.csv $P/${T}_pmc/write_size_counter_collection.csv
for i in 0 1 2; do cp $O/sq_${T}_$i/run_counter_collection.csv $P/${T}_sq/pass$i.csv; done
cp $O/pmc_traffic.json $P/pmc_traffic.json
cp $O/sq_counters.json $P/sq_counters.json
echo "collected $T"
