#!/bin/bash
# r03w: same-box A/B on C3: build_ab/cur.so (uniform pivot + contribution column order) and build_ab/w2.so (GICP at
# 2 waves per SIMD, no spills) against build_ab/upiv.so.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS="build_ab/cur.so" TESTK="icp or gicp" bash tools/c3_ab.sh > gpurun_out/r03w_ab1.txt 2>&1 || { tail -30 gpurun_out/r03w_ab1.txt; exit 1; }
cat gpurun_out/r03w_ab1.txt
LIBS="build_ab/upiv.so build_ab/w2.so build_ab/cur.so build_ab/upiv.so" TESTK=none bash tools/c3_ab.sh > gpurun_out/r03w_ab2.txt 2>&1 || { tail -30 gpurun_out/r03w_ab2.txt; exit 1; }; cat gpurun_out/r03w_ab2.txt
