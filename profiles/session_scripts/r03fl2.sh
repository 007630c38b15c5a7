#!/bin/bash
# r03fl2: -O2 (build_ab/o2.so) against -O3 (build_ab/base.so): GPU suite on o2, the default C2 bench alternating 4x,
# and C3 (bench_configs) once each.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PCORE_LIB=$PWD/build_ab/o2.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03fl2_pytest.log 2>&1 || { tail -30 gpurun_out/r03fl2_pytest.log; exit 1; }
echo "o2: $(tail -1 gpurun_out/r03fl2_pytest.log)"
for r in 1 2 3 4; do for L in base o2; do
  PCORE_LIB=$PWD/build_ab/$L.so timeout -k 10 300 python bench.py --no-cpu --c3-steps 0 --steps 40 > gpurun_out/r03fl2_${L}_$r.json 2> gpurun_out/r03fl2_${L}_$r.err || { tail -20 gpurun_out/r03fl2_${L}_$r.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r03fl2_${L}_$r.json')); print('$L', round(d['value']/1e6,3), round(d['ms_per_step'],4))"
done; done
for L in base o2; do
  PCORE_LIB=$PWD/build_ab/$L.so timeout -k 10 300 python tools/bench_configs.py --configs C3 --steps 5 2>/dev/null | cut -c1-150 || exit 1
done
