#!/bin/bash
# The source covariances folded into render_cloud_kernel against their own launch (PCORE_COV_SEPARATE=1): the
# covariance / GICP parity tests, then the bench's C3 leg alternating the two, twice.  TAG=<name> names the outputs.
set -o pipefail
OUT=gpurun_out/${TAG:-cf}
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "covariance or icp or gicp" \
  > $OUT/pytest_cov.log 2>&1 || { tail -40 $OUT/pytest_cov.log; exit 1; }
tail -1 $OUT/pytest_cov.log
for rep in 1 2; do
  for sep in 0 1; do
    if [ $sep = 1 ]; then export PCORE_COV_SEPARATE=1; else unset PCORE_COV_SEPARATE; fi
    timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --c3-steps 5 > $OUT/bench_sep${sep}_$rep.json 2> $OUT/bench_sep${sep}_$rep.err \
      || { tail -20 $OUT/bench_sep${sep}_$rep.err; exit 1; }
    python -c "import json; c=json.load(open('$OUT/bench_sep${sep}_$rep.json'))['c3']; print('separate=$sep C3 %.4g M  %.2f ms/step  icp stage %.2f  gicp %.2f' % (c['value']/1e6, c['ms_per_step'], c['gicp']['icp_stage_ms_per_step'], c['gicp']['gicp_ms_per_step']))"
  done
done
