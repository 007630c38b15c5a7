#!/bin/bash
# r03s2: same-box A/B on C3 of the two-query key scan (build_ab/scan2.so) against one scan per round (noscan2.so).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS="build_ab/scan2.so" TESTK="icp or gicp" bash tools/c3_ab.sh > gpurun_out/r03s2_ab1.txt 2>&1 || { tail -30 gpurun_out/r03s2_ab1.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r03s2_ab1.txt | cut -c1-200
LIBS="build_ab/noscan2.so build_ab/scan2.so build_ab/noscan2.so" TESTK=none bash tools/c3_ab.sh > gpurun_out/r03s2_ab2.txt 2>&1 || { tail -30 gpurun_out/r03s2_ab2.txt; exit 1; }; grep -v amdgpu.ids gpurun_out/r03s2_ab2.txt | cut -c1-200
