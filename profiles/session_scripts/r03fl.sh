#!/bin/bash
# r03fl: compiler-flag variants of the whole library (build_ab/{trk,o2,nopre}.so) against build_ab/base.so: the default
# C2 bench (two lanes), alternating with the base build.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in base trk base o2 base nopre base; do
  PCORE_LIB=$PWD/build_ab/$L.so timeout -k 10 300 python bench.py --no-cpu --c3-steps 0 --steps 40 > gpurun_out/r03fl_$L.json 2> gpurun_out/r03fl_$L.err || { tail -20 gpurun_out/r03fl_$L.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r03fl_$L.json')); print('$L', round(d['value']/1e6,3), round(d['ms_per_step'],4))"
done
