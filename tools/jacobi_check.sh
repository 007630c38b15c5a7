#!/bin/bash
# The thresholded Jacobi (the covariance spec's round-6 change, kernel and oracle in lockstep): the covariance / GICP
# parity tests, the GPU's GICP against the independent numpy chain on 1,000 candidates, and the covariance kernel's
# time per C3 call.  TAG names the output directory under gpurun_out/.
set -o pipefail
OUT=gpurun_out/${TAG:-jac}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "covariance or gicp or icp or recognizer" \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 900 python -u tools/gpu_vs_independent.py --poses-per-object 200 --out $OUT/gpu_vs_independent_1000.json > $OUT/gvi.log 2>&1 \
  || { tail -20 $OUT/gvi.log; exit 1; }
python -c "import json; d=json.load(open('$OUT/gpu_vs_independent_1000.json')); print({k: d[k] for k in ('equal_iteration_counts','over_1e-4','bit_identical_fraction','at_150')})"
KERNEL="covariance_cloud|gicp_kernel<" TAG=${TAG:-jac} LIBS="" bash tools/gicp_lib_ab.sh
