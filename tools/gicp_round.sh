#!/bin/bash
# GICP iteration round on one box: parity (icp / recognizer / metrics), A/B timing, phase profile.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out}
timeout -k 10 600 python -m pytest tests -q -m gpu ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/icp_pytest.log 2>&1 || { tail -30 $OUT/icp_pytest.log; exit 1; }
tail -1 $OUT/icp_pytest.log
if [ -n "$LIBS" ]; then KERNEL=gicp ARGS="--icp" bash tools/ab_time.sh || exit 1; fi
if [ -f build_ab/prof.so ]; then
  PCORE_LIB=$PWD/build_ab/prof.so timeout -k 10 300 python tools/gicp_phase_prof.py > $OUT/gicp_phase.log 2>&1 || { tail $OUT/gicp_phase.log; exit 1; }
  cat $OUT/gicp_phase.log
fi
