#!/bin/bash
# GICP parity tests, then C3 / C1 timing for the default build and alternative builds (LIBS="a.so b.so").
set -o pipefail
OUT=${OUT:-gpurun_out}; export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_recognizer.py -m gpu -x -q --timeout 300 --timeout-method thread -k "icp or localize" > $OUT/gicp_ab_pytest.log 2>&1 || { tail -30 $OUT/gicp_ab_pytest.log; exit 1; }
tail -1 $OUT/gicp_ab_pytest.log
timeout -k 10 300 python tools/bench_configs.py --configs ${CONFIGS:-C1,C3} --steps 3 | cut -c1-240 || exit 1
for L in $LIBS; do
  echo "== $L"
  PCORE_LIB=$PWD/$L timeout -k 10 300 python tools/bench_configs.py --configs ${CONFIGS:-C1,C3} --steps 3 | cut -c1-240 || exit 1
done
if [ -f build_ab/prof.so ]; then PCORE_LIB=$PWD/build_ab/prof.so timeout -k 10 200 python tools/gicp_phase_prof.py --c3 --poses 4000 || exit 1; fi
