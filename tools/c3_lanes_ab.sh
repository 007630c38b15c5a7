#!/bin/bash
# The bench's C3 leg with one and with two batches in flight (PCORE_BENCH_LANES), alternating, twice; the GICP parity
# tests first.  TAG names the outputs.
set -o pipefail
OUT=gpurun_out/${TAG:-cl}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTS:-icp or gicp}" \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for L in 1 2; do
    PCORE_BENCH_LANES=$L timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --c3-steps 6 > $OUT/bench_l${L}_$rep.json 2> $OUT/bench_l${L}_$rep.err \
      || { tail -20 $OUT/bench_l${L}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_l${L}_$rep.json')); c=d['c3']; print('lanes=$L C2 %.4g M  C3 %.4g M  %.2f ms/step  gicp %.2f ms  exit-off %.4g M' % (d['value']/1e6, c['value']/1e6, c['ms_per_step'], c['gicp']['gicp_ms_per_step'], c['gicp']['exit_off']['value']/1e6))"
  done
done
