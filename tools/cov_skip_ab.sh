set -o pipefail
OUT=gpurun_out/r06q; mkdir -p $OUT; export TMPDIR=/tmp
for L in perception_amd/libpcore.so build_ab/covskip1.so perception_amd/libpcore.so build_ab/covskip1.so; do
  T=$(basename $L .so)_$RANDOM
  PCORE_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ab_$T -o run -- python tools/prof_fused.py --c3 --icp --iters 3 > $OUT/ab_$T.log 2>&1 || { tail $OUT/ab_$T.log; exit 1; }
  echo "== $L $(grep -E 'covariance_cloud' $OUT/ab_$T/run_kernel_stats.csv | awk -F'\",' '{print $2}' | cut -d, -f1-3)"
done
