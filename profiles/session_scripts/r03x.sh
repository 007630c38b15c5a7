#!/bin/bash
# r03x: C1 GICP against the whole-scene grid with larger shell budgets (build_ab/sb*.so): C1 stats per build, then
# the dense / whole-scene GICP parity tests of the best candidates.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for B in 343 2197 9261 35937; do
  echo "== budget $B"
  PCORE_LIB=$PWD/build_ab/sb$B.so timeout -k 10 300 python -u tools/c1_gicp_stats.py 2>&1 | grep -v amdgpu.ids || exit 1
done
for B in 9261 35937; do
  PCORE_LIB=$PWD/build_ab/sb$B.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "whole_scene or dense or c1 or tabletop" > gpurun_out/r03x_pytest_$B.log 2>&1 || { tail -30 gpurun_out/r03x_pytest_$B.log; exit 1; }
  echo "sb$B: $(tail -1 gpurun_out/r03x_pytest_$B.log)"
done
