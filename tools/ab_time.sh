#!/bin/bash
# Interleaved A/B timing of alternative builds (PCORE_LIB) on one box: fused kernel mean duration.
set -o pipefail
OUT=${OUT:-gpurun_out}; export TMPDIR=/tmp
for round in 1 2 3; do
  for L in ${LIBS}; do
    n=$(basename $L .so)
    PCORE_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ab_${n}_$round -o run -- python tools/prof_fused.py --iters 5 ${ARGS} > $OUT/ab_${n}_$round.log 2>&1 || { tail $OUT/ab_${n}_$round.log; exit 1; }
    echo "$n r$round $(grep ${KERNEL:-fused_cost} $OUT/ab_${n}_$round/run_kernel_stats.csv | cut -d, -f3-4)"
  done
done
