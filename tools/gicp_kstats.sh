#!/bin/bash
# rocprofv3 kernel stats of C3 (evaluate_icp) under each PCORE_GICP_KERNEL pin in $PINS (default "n w").
set -o pipefail
OUT=${OUT:-gpurun_out}; export TMPDIR=/tmp; mkdir -p $OUT
for P in ${PINS:-n w}; do
  PCORE_GICP_KERNEL=$P timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/gk_$P -o run -- python tools/prof_fused.py --c3 --icp --iters 3 > $OUT/gk_$P.log 2>&1 || { tail $OUT/gk_$P.log; exit 1; }
  echo "== $P"; grep -E "gicp|fused_cost|render_cloud|covariance" $OUT/gk_$P/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
done
