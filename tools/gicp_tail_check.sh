#!/bin/bash
# The GICP launch's timeline (build_ab/tl.so: -DPCORE_GICP_TIMELINE) and phase clocks (build_ab/prof.so:
# -DPCORE_GICP_PROFILE) on C3, each under its own time limit.   TAG=<name> names the output directory.
set -o pipefail
OUT=gpurun_out/${TAG:-gt}
mkdir -p $OUT; export TMPDIR=/tmp
PCORE_LIB=$PWD/build_ab/tl.so timeout -k 10 300 python -u tools/gicp_timeline.py --out $OUT/gicp_timeline_c3.json > $OUT/timeline.log 2>&1 \
  || { tail -20 $OUT/timeline.log; exit 1; }
python -c "import json; d=json.load(open('$OUT/gicp_timeline_c3.json')); print({k: d[k] for k in d if k not in ('longest_poses', 'us_per_iteration_by_targets')}); print(d['longest_poses'][:4])"
PCORE_LIB=$PWD/build_ab/prof.so timeout -k 10 300 python -u tools/gicp_phase_prof.py --c3 > $OUT/gicp_phase_c3.txt 2>&1 || { tail -20 $OUT/gicp_phase_c3.txt; exit 1; }
cat $OUT/gicp_phase_c3.txt
