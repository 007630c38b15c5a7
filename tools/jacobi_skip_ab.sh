#!/bin/bash
# Round-6 timing study of the covariance kernel's Jacobi step (profiles/r06l2/): builds with a Numerical-Recipes skip of
# negligible rotations (then -DPCORE_JACOBI_SKIP=1 / 2, a study define since replaced by the spec's Eigen-JacobiSVD
# threshold in pcore_cov.h) and without the eigen-decomposition (-DPCORE_COV_SKIP=1), against the default build.
set -o pipefail
KERNEL=covariance_cloud TAG=r06l2 LIBS="build_ab/jskip1.so build_ab/jskip2.so build_ab/covskip1b.so" bash tools/gicp_lib_ab.sh
