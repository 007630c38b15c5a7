#!/bin/bash
# r03pf2: the default C2 bench (two lanes) with build_ab/pf1.so and build_ab/pf2.so, alternating, 3 rounds.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do for L in pf1 pf2; do
  PCORE_LIB=$PWD/build_ab/$L.so timeout -k 10 300 python bench.py --no-cpu --c3-steps 0 --steps 40 > gpurun_out/r03pf2_${L}_$r.json 2> gpurun_out/r03pf2_${L}_$r.err || { tail -20 gpurun_out/r03pf2_${L}_$r.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r03pf2_${L}_$r.json')); print('$L', round(d['value']/1e6,3), round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))"
done; done
