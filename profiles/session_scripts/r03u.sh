#!/bin/bash
# r03u: same-box A/B of the uniform LDLT pivot (build_ab/upiv.so) against HEAD's GICP (build_ab/gbase.so) on C3.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS="build_ab/upiv.so" TESTK="icp or gicp" bash tools/c3_ab.sh > gpurun_out/r03u_ab1.txt 2>&1 || { tail -30 gpurun_out/r03u_ab1.txt; exit 1; }
cat gpurun_out/r03u_ab1.txt
LIBS="build_ab/gbase.so build_ab/upiv.so build_ab/gbase.so" TESTK=none bash tools/c3_ab.sh > gpurun_out/r03u_ab2.txt 2>&1 || { tail -30 gpurun_out/r03u_ab2.txt; exit 1; }; cat gpurun_out/r03u_ab2.txt
