#!/bin/bash
# Launch timelines of C3's GICP call with the help board on and off (a -DPCORE_GICP_TIMELINE build, build_ab/tl_help.so:
# tools/build_variant.sh tl_help -DPCORE_GICP_TIMELINE), alternating; the longest chains with their start and end.
set -o pipefail
OUT=gpurun_out/${TAG:-help_tl}; mkdir -p $OUT; export TMPDIR=/tmp
for k in 1 2; do
for h in 1 0; do
PCORE_GICP_HELP=$h PCORE_LIB=$PWD/build_ab/tl_help.so timeout -k 10 300 python -u tools/gicp_timeline.py --out $OUT/tl_help${h}_$k.json > $OUT/tl_help${h}_$k.log 2>&1 || { tail -20 $OUT/tl_help${h}_$k.log; exit 1; }
python -c "
import json; d=json.load(open('$OUT/tl_help${h}_$k.json'))
print('help $h', {k: d[k] for k in ('span_us','busy_fraction','last_dequeue_us','tail_us','pose_us_max')})
print('longest', [(p['pose'], round(p['start_us']), round(p['start_us'] + p['us']), p['iterations'], p['points'], p['targets']) for p in d['longest_poses'][:5]])
print('last', [(p['pose'], round(p['start_us']), round(p['end_us']), p['iterations'], p['points'], p['targets']) for p in d['last_poses'][:6]])"
done
done
