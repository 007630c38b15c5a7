#!/bin/bash
# Same-box A/B of library builds on C3 (render + GICP + re-render): GICP/ICP parity tests per build, rocprofv3
# kernel stats of tools/prof_fused.py --c3 --icp, and bench_configs C3 throughput.  LIBS="build_ab/a.so ..."
# (TESTK=none skips the tests)
set -o pipefail
OUT=${OUT:-gpurun_out}; export TMPDIR=/tmp; mkdir -p $OUT
for L in $LIBS; do
  T=$(basename $L .so); export PCORE_LIB=$PWD/$L
  if [ "$TESTK" != "none" ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${TESTK:-icp}" > $OUT/pytest_c3_$T.log 2>&1 || { echo "FAIL $T"; tail -30 $OUT/pytest_c3_$T.log; exit 1; }
    echo "$T: $(tail -1 $OUT/pytest_c3_$T.log)"
  fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3ab_$T -o run -- python tools/prof_fused.py --c3 --icp --iters 3 > $OUT/c3ab_$T.log 2>&1 || { tail $OUT/c3ab_$T.log; exit 1; }
  python - <<PY
import csv
for r in csv.reader(open("$OUT/c3ab_$T/run_kernel_stats.csv")):
    if r[0] != "Name" and float(r[3]) > 100000: print("  %-50s %8.3f ms" % (r[0][:50], float(r[3]) / 1e6))
PY
  timeout -k 10 300 python tools/bench_configs.py --configs C3 --steps 5 | cut -c1-160 || exit 1
done
