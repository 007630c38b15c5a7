#!/bin/bash
# Phase clocks of gicp_kernel for all C3 poses (build_ab/prof.so) and for the poses of >= 300 source points only
# (build_ab/profbig.so: -DPCORE_GICP_PROF_MIN_NS=300), each under its own time limit.
set -o pipefail
OUT=gpurun_out/${TAG:-gpb}; mkdir -p $OUT; export TMPDIR=/tmp
for v in prof profbig; do
  PCORE_LIB=$PWD/build_ab/$v.so timeout -k 10 300 python -u tools/gicp_phase_prof.py --c3 > $OUT/gicp_phase_$v.txt 2>&1 || { tail -20 $OUT/gicp_phase_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $OUT/gicp_phase_$v.txt
done
