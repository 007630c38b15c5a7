#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel-trace summary.  Every GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-r01}
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $*"; }
step pytest && timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu_$TAG.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || exit $rc
step bench && timeout -k 10 600 python bench.py --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
if [ -n "$PROF" ]; then
  step rocprof && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python bench.py --steps 10 --warmup 2 --no-cpu > $OUT/prof_bench_$TAG.json 2> $OUT/prof_$TAG.err || { tail -20 $OUT/prof_$TAG.err; exit 1; }
  find $OUT/prof_$TAG -name "*stats*" | head
fi
