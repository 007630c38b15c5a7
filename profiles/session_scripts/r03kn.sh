#!/bin/bash
# r03kn: fused-kernel knobs at -O2 (build_ab/unr0.so: no 2x step unroll; build_ab/disc1.so: ring discard record) against
# the -O2 base: C2 bench alternating x2.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for L in base unr0 base disc1; do
  PCORE_LIB=$PWD/build_ab/$L.so timeout -k 10 300 python bench.py --no-cpu --c3-steps 0 --steps 40 > gpurun_out/r03kn_${L}_$r.json 2> gpurun_out/r03kn_${L}_$r.err || { tail -20 gpurun_out/r03kn_${L}_$r.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r03kn_${L}_$r.json')); print('$L', round(d['value']/1e6,3), round(d['ms_per_step'],4))"
done; done
