#!/bin/bash
# Same-box A/B of (library, environment) pairs on the C2 bench and (optionally) C5:
#   RUNS="base.so: t7.so: t7.so:PCORE_FUSED_TIER=0" tools/env_ab.sh   (libraries under build_ab/)
# TESTK: pytest -k expression run once per distinct library first (parity of the variant).
set -o pipefail
OUT=${OUT:-gpurun_out}; export TMPDIR=/tmp; mkdir -p $OUT
if [ -n "$TESTK" ]; then
  for L in $(for r in $RUNS; do echo ${r%%:*}; done | sort -u); do
    PCORE_LIB=$PWD/build_ab/$L timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$TESTK" > $OUT/pytest_ab_$L.log 2>&1 || { echo "FAIL $L"; tail -30 $OUT/pytest_ab_$L.log; exit 1; }
    echo "$L: $(tail -1 $OUT/pytest_ab_$L.log)"
  done
fi
for rep in $(seq 1 ${REPS:-2}); do
  for r in $RUNS; do
    L=${r%%:*}; E=${r#*:}
    env PCORE_LIB=$PWD/build_ab/$L $E timeout -k 10 300 python bench.py --no-cpu ${BENCH_ARGS} > $OUT/envab.json 2> $OUT/envab.err || { tail -20 $OUT/envab.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/envab.json')); print('$r: %.4gM poses/s  kernel %.4f ms' % (d['value']/1e6, d['roofline']['kernel_ms']))"
    if [ -n "$C5" ]; then
      env PCORE_LIB=$PWD/build_ab/$L $E timeout -k 10 300 python tools/bench_configs.py --configs C5 --steps 5 | cut -c1-150 || exit 1
    fi
  done
done
