#!/bin/bash
# r03y: the adaptive shell budget (build_ab/adapt.so): GICP parity tests, C1 / C3 GICP times; C1 phase clocks of
# gicp_wide_kernel (build_ab/prof.so).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PCORE_LIB=$PWD/build_ab/adapt.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "icp or gicp or whole_scene or dense or tabletop" > gpurun_out/r03y_pytest.log 2>&1 || { tail -30 gpurun_out/r03y_pytest.log; exit 1; }
echo "adapt: $(tail -1 gpurun_out/r03y_pytest.log)"
PCORE_LIB=$PWD/build_ab/adapt.so timeout -k 10 300 python -u tools/c1_gicp_stats.py 2>&1 | grep -v amdgpu.ids || exit 1
PCORE_LIB=$PWD/build_ab/adapt.so timeout -k 10 300 python -u tools/bench_configs.py --configs C1,C3 --steps 5 2>&1 | grep -v amdgpu.ids | cut -c1-220 || exit 1
PCORE_LIB=$PWD/build_ab/prof.so timeout -k 10 300 python -u tools/c1_phase_prof.py 2>&1 | grep -v amdgpu.ids || exit 1
