#!/bin/bash
# gicp_kernel's time per C3 call (rocprofv3 kernel trace over tools/prof_fused.py --c3 --icp, 3 calls) for the default
# build and the builds in LIBS, alternating twice.  TAG names the output directory under gpurun_out/.
set -o pipefail
OUT=gpurun_out/${TAG:-libab}; mkdir -p $OUT; export TMPDIR=/tmp
for k in 1 2; do
for L in perception_amd/libpcore.so $LIBS; do
  T=$(basename $L .so)_$RANDOM
  PCORE_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ab_$T -o run -- python tools/prof_fused.py --c3 --icp --iters 3 > $OUT/ab_$T.log 2>&1 || { tail $OUT/ab_$T.log; exit 1; }
  echo "== $L $(grep -E "${KERNEL:-gicp_kernel<}" $OUT/ab_$T/run_kernel_stats.csv | awk -F'",' '{print $2}' | cut -d, -f1-3)"
done
done
