#!/bin/bash
# The threshold k-NN with the cloud's points in LDS (-DPCORE_THR_LDS_PTS=N builds in LIBS): the covariance parity tests
# against each build, then covariance_cloud_kernel's time per C3 call alternating with the default build.
set -o pipefail
OUT=gpurun_out/${TAG:-covlds}; mkdir -p $OUT; export TMPDIR=/tmp
for L in $LIBS; do
  PCORE_LIB=$PWD/$L timeout -k 10 600 python -u -m pytest tests/test_gpu_covariances.py tests/test_gpu_fullsize.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "covariance or threshold or c3_scene_icp" > $OUT/pytest_$(basename $L .so).log 2>&1 \
    || { tail -30 $OUT/pytest_$(basename $L .so).log; exit 1; }
  echo "$L: $(tail -1 $OUT/pytest_$(basename $L .so).log)"
done
KERNEL=covariance_cloud TAG=${TAG:-covlds} LIBS="$LIBS" bash tools/gicp_lib_ab.sh
