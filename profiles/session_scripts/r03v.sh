#!/bin/bash
# r03v: same-box A/B of the round-1 trial-error prefetch (build_ab/pref.so) against build_ab/upiv.so on C3.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS="build_ab/pref.so" TESTK="icp or gicp" bash tools/c3_ab.sh > gpurun_out/r03v_ab1.txt 2>&1 || { tail -30 gpurun_out/r03v_ab1.txt; exit 1; }
cat gpurun_out/r03v_ab1.txt
LIBS="build_ab/upiv.so build_ab/pref.so build_ab/upiv.so" TESTK=none bash tools/c3_ab.sh > gpurun_out/r03v_ab2.txt 2>&1 || { tail -30 gpurun_out/r03v_ab2.txt; exit 1; }; cat gpurun_out/r03v_ab2.txt
