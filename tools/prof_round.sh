#!/bin/bash
# Where the time goes: fused-kernel ablations (PCORE_DEBUG_SKIP) and the C3 kernel breakdown.
set -o pipefail
OUT=${OUT:-gpurun_out}; export TMPDIR=/tmp; TAG=${TAG:-pr}
mkdir -p $OUT
OUT=$OUT bash tools/ablate.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3_$TAG -o run -- python tools/bench_configs.py --configs C3 --steps 2 > $OUT/c3_$TAG.log 2>&1 || { tail $OUT/c3_$TAG.log; exit 1; }
cut -d, -f1-5 $OUT/c3_$TAG/run_kernel_stats.csv | head -12
