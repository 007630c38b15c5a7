#!/bin/bash
# Full GPU session: parity tests, smoke, the counter passes that the bench line's roofline reads (two PMC
# passes FETCH_SIZE / WRITE_SIZE -> profiles/pmc_traffic.json, three SQ passes -> profiles/sq_counters.json,
# both tagged with the kernel-source digest; four SQ passes over gicp_kernel on C3 -> profiles/sq_counters_gicp.json,
# tagged with the GICP-source digest), the bench itself, and the rocprofv3 kernel-trace summary of the
# same bench command.  The folded json files are copied to $OUT (gpurun_out/ comes back; profiles/ on the box
# does not).  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out}; TAG=${TAG:-r04}
mkdir -p $OUT; export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  echo "== pytest"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1 || { tail -30 $OUT/pytest_gpu_$TAG.log; exit 1; }
  tail -3 $OUT/pytest_gpu_$TAG.log
  echo "== smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { tail -30 $OUT/smoke_$TAG.log; exit 1; }
  cat $OUT/smoke_$TAG.log
fi
if [ -z "$SKIP_PMC" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "== pmc $C"
    timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_${TAG}_$C -o run -- python bench.py --steps 3 --warmup 1 --no-cpu > $OUT/pmc_${TAG}_$C.json 2> $OUT/pmc_${TAG}_$C.err || { tail -20 $OUT/pmc_${TAG}_$C.err; exit 1; }
  done
  python tools/pmc_traffic.py $OUT/pmc_${TAG}_FETCH_SIZE/run_counter_collection.csv $OUT/pmc_${TAG}_WRITE_SIZE/run_counter_collection.csv profiles/pmc_traffic.json || exit 1
  cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
  echo "== sq counters"
  OUT=$OUT TAG=sq_$TAG bash tools/sq_counters.sh || exit 1
  python tools/sq_json.py $OUT sq_$TAG 10000 || exit 1
  cp profiles/sq_counters.json $OUT/sq_counters.json
  echo "== sq counters, GICP (C3)"
  OUT=$OUT TAG=sqg_$TAG bash tools/sq_gicp.sh || exit 1
  python tools/sq_gicp_json.py $OUT sqg_$TAG || exit 1
  cp profiles/sq_counters_gicp.json $OUT/sq_counters_gicp.json
fi
echo "== bench"
timeout -k 10 600 python bench.py ${BENCH_ARGS} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
echo "== rocprof stats"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python bench.py --no-cpu ${BENCH_ARGS} > $OUT/prof_bench_$TAG.json 2> $OUT/prof_$TAG.err || { tail -20 $OUT/prof_$TAG.err; exit 1; }
cat $OUT/prof_bench_$TAG.json
python tools/trace_busy.py $OUT/prof_$TAG/run_kernel_trace.csv --last ${STEPS:-20} --sq profiles/sq_counters.json --out $OUT/trace_busy_$TAG.json --stats-out $OUT/c2_kernel_stats_$TAG.csv || exit 1
find $OUT -path "*_$TAG*" -name "*.csv" | head -20
