set -o pipefail
OUT=gpurun_out/r06i; mkdir -p $OUT; export TMPDIR=/tmp
for hm in 8 0; do
PCORE_GICP_HEAVY_MAX=$hm PCORE_LIB=$PWD/build_ab/tl.so timeout -k 10 300 python -u tools/gicp_timeline.py --out $OUT/tl_h$hm.json > $OUT/tl_h$hm.log 2>&1 || { tail -20 $OUT/tl_h$hm.log; exit 1; }
python -c "import json; d=json.load(open('$OUT/tl_h$hm.json')); print('heavy_max $hm', {k: d[k] for k in ('span_us','busy_fraction','last_dequeue_us','tail_us','pose_us_max')}); print([(p['pose'], p['us'], p['iterations'], p['points'], p['start_us']) for p in d['longest_poses'][:6]])"
done
