#!/bin/bash
# One GPU-box pass over the GICP cycle exit: the GICP GPU tests, the bench (its C3 leg carries the exit on/off A/B)
# and the parity sweep's exit on/off comparison on 5,000 C3 candidates.  Every GPU step has its own time limit; the
# chain stops at the first failure.   TAG=<name> names the output directory under gpurun_out/.
set -o pipefail
OUT=gpurun_out/${TAG:-gx}
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTS:-gicp or icp or covariance}" \
  > $OUT/pytest_gicp.log 2>&1 || { tail -40 $OUT/pytest_gicp.log; exit 1; }
tail -2 $OUT/pytest_gicp.log
timeout -k 10 400 python -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python - "$OUT/bench.json" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
c = d["c3"]
print("C2 %.4g M poses/s; C3 %.4g M poses/s %.2f ms/step, gicp %.2f ms" % (
    d["value"] / 1e6, c["value"] / 1e6, c["ms_per_step"], c["gicp"]["gicp_ms_per_step"]))
print(json.dumps(c["gicp"]))
EOF
[ -n "$NO_SWEEP" ] && exit 0
timeout -k 10 600 python -u tools/parity_sweep.py --batches 0 --icp ${ICP:-5000} --out $OUT/parity_sweep_icp.json \
  > $OUT/sweep.log 2>&1 || { tail -20 $OUT/sweep.log; exit 1; }
cat $OUT/parity_sweep_icp.json
