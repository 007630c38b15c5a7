#!/bin/bash
# One A/B session: parity subset of every variant in $LIBS (pytest -k "$TESTK"), then tools/lib_ab.sh over them,
# then per-phase clocks of the profile builds in $PROFLIBS.
set -o pipefail
OUT=${OUT:-gpurun_out}; export TMPDIR=/tmp; mkdir -p $OUT
for L in $LIBS; do
  T=$(basename $L .so)
  if [ -n "$TESTK" ]; then
    PCORE_LIB=$PWD/$L timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$TESTK" > $OUT/pytest_$T.log 2>&1 || { echo "FAIL $T"; tail -30 $OUT/pytest_$T.log; exit 1; }
    echo "$T: $(tail -1 $OUT/pytest_$T.log)"
  fi
done
LIBS="$LIBS" bash tools/lib_ab.sh || exit 1
for L in $PROFLIBS; do
  echo "== phases $(basename $L .so)"
  PCORE_LIB=$PWD/$L timeout -k 10 300 python tools/fused_phase_prof.py || exit 1
done
