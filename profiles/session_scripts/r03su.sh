#!/bin/bash
# r03su: GICP key-scan unroll at -O2 (build_ab/su2.so, su8.so) against the base (4 quad pairs per trip), C3, alternating.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS="build_ab/base.so build_ab/su2.so build_ab/base.so build_ab/su8.so build_ab/base.so" TESTK=none bash tools/c3_ab.sh > gpurun_out/r03su.txt 2>&1 || { tail -30 gpurun_out/r03su.txt; exit 1; }
grep -E "gicp_kernel|C3" gpurun_out/r03su.txt | cut -c1-160
