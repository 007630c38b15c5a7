#!/bin/bash
# scan_quads2 with one compare per pair of quads per chain (-DPCORE_SCAN_PAIRQ=1 builds in LIBS): the GICP parity tests
# against each build, then gicp_kernel's time per C3 call alternating with the default build.
set -o pipefail
OUT=gpurun_out/${TAG:-pairq}; mkdir -p $OUT; export TMPDIR=/tmp
for L in $LIBS; do
  PCORE_LIB=$PWD/$L timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "gicp or icp" > $OUT/pytest_$(basename $L .so).log 2>&1 || { tail -30 $OUT/pytest_$(basename $L .so).log; exit 1; }
  echo "$L: $(tail -1 $OUT/pytest_$(basename $L .so).log)"
done
TAG=${TAG:-pairq} LIBS="$LIBS" bash tools/gicp_lib_ab.sh
