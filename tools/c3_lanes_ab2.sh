#!/bin/bash
# The bench's C3 leg with one and two batches in flight (PCORE_BENCH_C3_LANES), alternating twice on one box.
set -o pipefail
OUT=gpurun_out/${TAG:-c3l}; mkdir -p $OUT; export TMPDIR=/tmp
for k in 1 2; do
for L in 1 2; do
  PCORE_BENCH_C3_LANES=$L timeout -k 10 400 python -u bench.py --no-cpu --steps 5 > $OUT/bench_l${L}_$k.json 2> $OUT/bench_l${L}_$k.err || { tail -20 $OUT/bench_l${L}_$k.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_l${L}_$k.json').read().strip().splitlines()[-1]); c=d['c3']; print('lanes $L', round(c['value']/1e6,3), 'M', round(c['ms_per_step'],2), 'ms', 'gicp', round(c['gicp']['gicp_ms_per_step'],2))"
done
done
