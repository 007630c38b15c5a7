#!/bin/bash
# r03kn2: PCORE_RING_DISCARD=1 (build_ab/disc1.so) against the -O2 base: GPU suite on disc1, C2 bench alternating x4.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PCORE_LIB=$PWD/build_ab/disc1.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03kn2_pytest.log 2>&1 || { tail -30 gpurun_out/r03kn2_pytest.log; exit 1; }
echo "disc1: $(tail -1 gpurun_out/r03kn2_pytest.log)"
for r in 1 2 3 4; do for L in base disc1; do
  PCORE_LIB=$PWD/build_ab/$L.so timeout -k 10 300 python bench.py --no-cpu --c3-steps 0 --steps 40 > gpurun_out/r03kn2_${L}_$r.json 2> gpurun_out/r03kn2_${L}_$r.err || { tail -20 gpurun_out/r03kn2_${L}_$r.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r03kn2_${L}_$r.json')); print('$L', round(d['value']/1e6,3), round(d['ms_per_step'],4))"
done; done
