#!/bin/bash
# fused-kernel pose windows: parity tests, then C2 kernel times and C2/C3/C5 throughput per LDS tile tier
# (PCORE_FUSED_TIER; "auto" = the histogram choice, 5 = whole image)
set -o pipefail
OUT=${OUT:-gpurun_out}; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/win_pytest.log 2>&1 || { tail -40 $OUT/win_pytest.log; exit 1; }
tail -1 $OUT/win_pytest.log
for T in ${TIERS:-auto 5}; do
  if [ "$T" = auto ]; then unset PCORE_FUSED_TIER; else export PCORE_FUSED_TIER=$T; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/win_$T -o run -- python tools/prof_fused.py --iters 5 ${ARGS} > $OUT/win_$T.log 2>&1 || { tail $OUT/win_$T.log; exit 1; }
  echo "tier=$T"; grep -E "fused_cost" $OUT/win_$T/run_kernel_stats.csv | cut -d, -f1-5
  if [ -n "$CONFIGS" ]; then timeout -k 10 300 python tools/bench_configs.py --configs $CONFIGS --steps 3 | cut -c1-200 || exit 1; fi
done
