#!/bin/bash
# Per-kernel GPU time of alternative library builds on C3 (render + covariances + GICP + re-render), one rocprofv3
# kernel-trace pass per build: LIBS="default build_ab/a.so ..." KERNELS="covariance_kernel gicp_kernel" tools/kernel_ab.sh
set -o pipefail
OUT=${OUT:-gpurun_out}; export TMPDIR=/tmp; mkdir -p $OUT
for L in $LIBS; do
  T=$(basename $L .so)
  if [ "$L" = default ]; then unset PCORE_LIB; else export PCORE_LIB=$PWD/$L; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kab_$T -o run -- python tools/prof_fused.py --c3 --icp --iters 3 > $OUT/kab_$T.log 2>&1 || { tail $OUT/kab_$T.log; exit 1; }
  python - "$OUT/kab_$T/run_kernel_stats.csv" "$T" "${KERNELS:-covariance_kernel gicp_kernel}" <<'PY'
import csv, sys
path, tag, keys = sys.argv[1], sys.argv[2], sys.argv[3].split()
for r in csv.DictReader(open(path)):
    if any(k in r["Name"] for k in keys):
        print(f"{tag:10s} {r['Name'][:60]:60s} calls {r['Calls']:>4s} avg {float(r['AverageNs']) / 1e6:8.3f} ms")
PY
done
