#!/bin/bash
# r03k: DPP reduction of the normal equations (3 and 4 waves per SIMD) vs HEAD on C3; then GICP SQ passes at
# HEAD and the recognizer end-to-end timing (tools/r03i.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="build_ab/base.so build_ab/dpp.so build_ab/dpp4.so build_ab/base.so build_ab/dpp.so build_ab/dpp4.so" TESTK="icp" bash tools/c3_ab.sh > gpurun_out/r03k_c3ab.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03k_c3ab.txt | cut -c1-150; [ $rc -eq 0 ] || exit $rc
bash tools/r03i.sh
