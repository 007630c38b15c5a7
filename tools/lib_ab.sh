#!/bin/bash
# A/B of alternative library builds (LIBS="build_ab/a.so build_ab/b.so"): kernel times (rocprofv3 stats of
# tools/prof_fused.py $ARGS, rows matching $KERNELS) and bench_configs throughput ($CONFIGS, default C2,C5).
set -o pipefail
OUT=${OUT:-gpurun_out}; export TMPDIR=/tmp
for L in $LIBS; do
  T=$(basename $L .so)
  export PCORE_LIB=$PWD/$L
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ab_$T -o run -- python tools/prof_fused.py --iters 5 ${ARGS} > $OUT/ab_$T.log 2>&1 || { tail $OUT/ab_$T.log; exit 1; }
  echo "== $T"; grep -E "${KERNELS:-fused_cost}" $OUT/ab_$T/run_kernel_stats.csv | cut -d, -f1-4
  timeout -k 10 300 python tools/bench_configs.py --configs ${CONFIGS:-C2,C5} --steps 5 | cut -c1-170 || exit 1
done
