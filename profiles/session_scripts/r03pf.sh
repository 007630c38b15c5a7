#!/bin/bash
# r03pf: the fused kernel's two-step-ahead prefetch (build_ab/pf2.so) against one step ahead (build_ab/pf1.so): the
# whole GPU suite on pf2, then same-box kernel times and C2 / C5 throughput, alternating.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PCORE_LIB=$PWD/build_ab/pf2.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03pf_pytest.log 2>&1 || { tail -30 gpurun_out/r03pf_pytest.log; exit 1; }
echo "pf2: $(tail -1 gpurun_out/r03pf_pytest.log)"
LIBS="build_ab/pf1.so build_ab/pf2.so build_ab/pf1.so build_ab/pf2.so" CONFIGS=C2,C5 bash tools/lib_ab.sh > gpurun_out/r03pf_ab.txt 2>&1 || { tail -30 gpurun_out/r03pf_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r03pf_ab.txt | cut -c1-200
