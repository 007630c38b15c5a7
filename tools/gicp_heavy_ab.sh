#!/bin/bash
# gicp_kernel's heavy poses (one 4-wave workgroup each) against none (PCORE_GICP_HEAVY_MAX=0): the GICP parity tests,
# then the bench's C3 leg alternating the two, twice, and the launch timeline with them.  TAG names the outputs.
set -o pipefail
OUT=gpurun_out/${TAG:-gh}
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTS:-icp or gicp or covariance}" \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for hm in default 0; do
    if [ $hm = default ]; then unset PCORE_GICP_HEAVY_MAX; else export PCORE_GICP_HEAVY_MAX=$hm; fi
    timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --c3-steps 5 > $OUT/bench_h${hm}_$rep.json 2> $OUT/bench_h${hm}_$rep.err \
      || { tail -20 $OUT/bench_h${hm}_$rep.err; exit 1; }
    python -c "import json; c=json.load(open('$OUT/bench_h${hm}_$rep.json'))['c3']; print('heavy_max=$hm C3 %.4g M  %.2f ms/step  gicp %.2f ms' % (c['value']/1e6, c['ms_per_step'], c['gicp']['gicp_ms_per_step']))"
  done
done
unset PCORE_GICP_HEAVY_MAX
PCORE_LIB=$PWD/build_ab/tl.so timeout -k 10 300 python -u tools/gicp_timeline.py --out $OUT/gicp_timeline_c3.json > $OUT/timeline.log 2>&1 \
  || { tail -20 $OUT/timeline.log; exit 1; }
python -c "import json; d=json.load(open('$OUT/gicp_timeline_c3.json')); print({k: d[k] for k in ('span_us','busy_fraction','last_dequeue_us','tail_us','pose_us_max','poses_run_150')}); print(d['longest_poses'][:4])"
