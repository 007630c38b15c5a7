#!/bin/bash
# r03z: the cell-list fallback of the whole-scene / dense GICP search (build_ab/clist.so) against the adaptive shell
# budget (build_ab/adapt.so): parity tests, C1 GICP stats and phases, C3 timing.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PCORE_LIB=$PWD/build_ab/clist.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "icp or gicp or whole_scene or dense or tabletop" > gpurun_out/r03z_pytest.log 2>&1 || { tail -30 gpurun_out/r03z_pytest.log; exit 1; }
echo "clist: $(tail -1 gpurun_out/r03z_pytest.log)"
for L in clist adapt clist; do
  echo "== $L"; PCORE_LIB=$PWD/build_ab/$L.so timeout -k 10 300 python -u tools/c1_gicp_stats.py 2>&1 | grep -v amdgpu.ids || exit 1
done
PCORE_LIB=$PWD/build_ab/clistprof.so timeout -k 10 300 python -u tools/c1_phase_prof.py 2>&1 | grep -v amdgpu.ids || exit 1
LIBS="build_ab/adapt.so build_ab/clist.so" TESTK=none bash tools/c3_ab.sh > gpurun_out/r03z_c3.txt 2>&1 || { tail -30 gpurun_out/r03z_c3.txt; exit 1; }; grep -v amdgpu.ids gpurun_out/r03z_c3.txt | cut -c1-200
