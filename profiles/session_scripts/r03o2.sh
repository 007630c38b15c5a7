#!/bin/bash
# r03o2: occupancy bitmaps in the grid shell search (build_ab/occ.so) against HEAD (build_ab/adapt.so): GICP /
# large-segment parity tests, C1 GICP stats and phases, C3 timing.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PCORE_LIB=$PWD/build_ab/occ.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "icp or gicp or whole_scene or dense or tabletop or far_queries" > gpurun_out/r03o2_pytest.log 2>&1 || { tail -30 gpurun_out/r03o2_pytest.log; exit 1; }
echo "occ: $(tail -1 gpurun_out/r03o2_pytest.log)"
for L in occ adapt occ; do
  echo "== $L"; PCORE_LIB=$PWD/build_ab/$L.so timeout -k 10 300 python -u tools/c1_gicp_stats.py 2>&1 | grep -v amdgpu.ids || exit 1
done
PCORE_LIB=$PWD/build_ab/occprof.so timeout -k 10 300 python -u tools/c1_phase_prof.py 2>&1 | grep -v amdgpu.ids || exit 1
LIBS="build_ab/adapt.so build_ab/occ.so" TESTK=none bash tools/c3_ab.sh > gpurun_out/r03o2_c3.txt 2>&1 || { tail -30 gpurun_out/r03o2_c3.txt; exit 1; }; grep -v amdgpu.ids gpurun_out/r03o2_c3.txt | cut -c1-200
