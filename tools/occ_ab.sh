#!/bin/bash
# A/B of fused-kernel occupancy builds: for each "lib:granule" in $RUNS, the C2 kernel time at 10,000 poses
# (tools/tail_probe.py, HIP events) and bench_configs throughput of $CONFIGS (default C2,C5).
set -o pipefail
OUT=${OUT:-gpurun_out}
for R in $RUNS; do
  L=${R%%:*}; G=${R##*:}
  export PCORE_LIB=$PWD/$L PCORE_LDS_GRANULE=$G
  echo "== $L granule $G"
  timeout -k 10 120 python tools/tail_probe.py --sizes 10000,20000 --iters 20 2> $OUT/occ_ab.err || { tail $OUT/occ_ab.err; exit 1; }
  timeout -k 10 300 python tools/bench_configs.py --configs ${CONFIGS:-C2,C5} --steps 5 2>> $OUT/occ_ab.err | cut -c1-150 || { tail $OUT/occ_ab.err; exit 1; }
done
