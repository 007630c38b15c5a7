#!/bin/bash
# Kernel time of the fused kernel under PCORE_DEBUG_SKIP ablations (rocprofv3 kernel-trace stats).
set -o pipefail
OUT=${OUT:-gpurun_out}; export TMPDIR=/tmp
# the production build ignores PCORE_DEBUG_SKIP: these passes load an ablation build
# (tools/build_variant.sh ablate -DPCORE_DEBUG_SKIP_RT=1, made here on the CPU beforehand)
export PCORE_LIB=${PCORE_LIB:-$PWD/build_ab/ablate.so}
[ -f "$PCORE_LIB" ] || { echo "missing $PCORE_LIB (tools/build_variant.sh ablate -DPCORE_DEBUG_SKIP_RT=1)"; exit 1; }
for M in 0 1 2 3 4 7 15; do
  PCORE_DEBUG_SKIP=$M timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/abl_$M -o run -- python tools/prof_fused.py --iters 5 > $OUT/abl_$M.log 2>&1 || { tail $OUT/abl_$M.log; exit 1; }
  echo "skip=$M $(grep fused_cost $OUT/abl_$M/run_kernel_stats.csv | cut -d, -f2-5)"
done
