#!/bin/bash
# r03j: multi-round correspondence scan (R rounds of queries per pass over the quads) vs HEAD, C3 A/B + phases.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="build_ab/base.so build_ab/multi2.so build_ab/multi1.so build_ab/multi4.so build_ab/multi2.so build_ab/base.so" TESTK="icp" bash tools/c3_ab.sh > gpurun_out/r03j_c3ab.txt 2>&1 && \
PCORE_LIB=$PWD/build_ab/gprofm.so timeout -k 10 200 python -u tools/gicp_phase_prof.py --c3 > gpurun_out/r03j_phase.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03j_c3ab.txt | cut -c1-150; cat gpurun_out/r03j_phase.txt; exit $rc
