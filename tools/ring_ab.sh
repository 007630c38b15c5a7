#!/bin/bash
# GPU parity tests of the current build, the flush statistics (build_ab/fst.so, when built), then a same-box A/B of
# build_ab/old.so against build_ab/new.so (tools/occ_ab.sh, configs C2, C3, C5).
set -o pipefail
OUT=${OUT:-gpurun_out}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_ring.log 2>&1 || { tail -30 $OUT/pytest_ring.log; exit 1; }
tail -2 $OUT/pytest_ring.log
if [ -f build_ab/fst.so ]; then PCORE_LIB=$PWD/build_ab/fst.so timeout -k 10 100 python tools/flush_stats.py 2> $OUT/fst.err || exit 1; fi
RUNS="build_ab/old.so:1280 build_ab/new.so:1280 build_ab/old.so:1280 build_ab/new.so:1280" CONFIGS=C2,C3,C5 bash tools/occ_ab.sh
