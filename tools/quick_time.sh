#!/bin/bash
# fused-kernel time (rocprofv3 kernel stats) + the C2 parity tests
set -o pipefail
OUT=${OUT:-gpurun_out}; export TMPDIR=/tmp; TAG=${TAG:-qt}
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -x -k "evaluate or sampled or fixture or edge" > $OUT/${TAG}_pytest.log 2>&1 || { tail -30 $OUT/${TAG}_pytest.log; exit 1; }
tail -1 $OUT/${TAG}_pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG} -o run -- python tools/prof_fused.py --iters 5 ${ARGS} > $OUT/${TAG}.log 2>&1 || { tail $OUT/${TAG}.log; exit 1; }
grep -E "fused_cost|gicp|covariance|render_cloud" $OUT/${TAG}/run_kernel_stats.csv | cut -d, -f1-5
