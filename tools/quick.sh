#!/bin/bash
# Quick GPU iteration: (optional) GPU parity suite, then the bench without the CPU baselines.  Every GPU step
# has its own time limit; the chain stops at the first failure.   TESTS=1 / TESTS=<pytest -k expr>
set -o pipefail
OUT=${OUT:-gpurun_out}; TAG=${TAG:-q}
mkdir -p $OUT; export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  K=""; [ "$TESTS" != "1" ] && K="-k $TESTS"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $K > $OUT/pytest_$TAG.log 2>&1 || { tail -30 $OUT/pytest_$TAG.log; exit 1; }
  tail -2 $OUT/pytest_$TAG.log
fi
for i in $(seq 1 ${BENCH_REPS:-1}); do
  timeout -k 10 300 python bench.py --no-cpu ${BENCH_ARGS} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -20 $OUT/bench_$TAG.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$TAG.json')); print('value %.4gM poses/s  kernel %.4f ms' % (d['value']/1e6, d['roofline']['kernel_ms']))"
done
