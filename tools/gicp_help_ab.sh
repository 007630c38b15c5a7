#!/bin/bash
# The GICP help board on the GPU box: the GICP / help parity tests, then gicp_kernel's time per C3 call (rocprofv3
# kernel trace, tools/prof_fused.py --c3 --icp) with the board on, off (PCORE_GICP_HELP=0, same build) and for the
# build without it (build_ab/base.so, LIBS to override), alternating; then the bench's C3 leg.  TAG names the output
# directory under gpurun_out/.  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
OUT=gpurun_out/${TAG:-help}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s \
  -k "${TESTS:-help or gicp or icp or covariance}" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
grep -E "passed|failed|help board" $OUT/pytest.log | tail -4
run() {  # $1 label, $2 lib, $3 PCORE_GICP_HELP
  T=$1_$RANDOM
  PCORE_GICP_HELP=$3 PCORE_LIB=$PWD/$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ab_$T \
    -o run -- python tools/prof_fused.py --c3 --icp --iters 3 > $OUT/ab_$T.log 2>&1 || { tail $OUT/ab_$T.log; return 1; }
  echo "== $1: $(grep 'gicp_kernel<' $OUT/ab_$T/run_kernel_stats.csv | awk -F'",' '{print $2}' | cut -d, -f1-3)"
}
for k in 1 2; do
  run help perception_amd/libpcore.so 1 || exit 1
  run off perception_amd/libpcore.so 0 || exit 1
  run base ${BASE:-build_ab/base.so} 1 || exit 1
done
timeout -k 10 400 python -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c = d["c3"]
print("C2 %.4g M poses/s; C3 %.4g M poses/s %.2f ms/step, gicp %.2f ms" % (
    d["value"] / 1e6, c["value"] / 1e6, c["ms_per_step"], c["gicp"]["gicp_ms_per_step"]))
PY
