#!/bin/bash
# Parity at scale at the final build: the covariance GPU tests, then tools/parity_sweep.py -- 100,000 random poses at
# 640x480 and 20,000 at 1280x720 against the oracle, and 5,000 C3-style GICP candidates with the cycle exit on and off.
set -o pipefail
OUT=gpurun_out/${TAG:-par}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_covariances.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_cov.log 2>&1 || { tail -30 $OUT/pytest_cov.log; exit 1; }
tail -1 $OUT/pytest_cov.log
timeout -k 10 1000 python -u tools/parity_sweep.py --icp 5000 --out $OUT/parity_sweep.json > $OUT/sweep.log 2>&1 \
  || { tail -20 $OUT/sweep.log; exit 1; }
python -c "import json; d=json.load(open('$OUT/parity_sweep.json')); print(json.dumps(d)[:1500])"
