#!/bin/bash
# The clouds' covariances by the threshold k-NN (default) against the brute-force kernel (PCORE_COV_BRUTE=1): the
# covariance and GICP parity tests, then the bench's C3 leg alternating the two, twice.  TAG names the outputs.
set -o pipefail
OUT=gpurun_out/${TAG:-ct}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTS:-covariance or icp or gicp}" \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for b in 0 1; do
    if [ $b = 1 ]; then export PCORE_COV_BRUTE=1; else unset PCORE_COV_BRUTE; fi
    timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --c3-steps 5 > $OUT/bench_b${b}_$rep.json 2> $OUT/bench_b${b}_$rep.err \
      || { tail -20 $OUT/bench_b${b}_$rep.err; exit 1; }
    python -c "import json; c=json.load(open('$OUT/bench_b${b}_$rep.json'))['c3']; g=c['gicp']; print('brute=$b C3 %.4g M  %.2f ms/step  icp stage %.2f  gicp %.2f' % (c['value']/1e6, c['ms_per_step'], g['icp_stage_ms_per_step'], g['gicp_ms_per_step']))"
  done
done
