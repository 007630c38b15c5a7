#!/bin/bash
# r03p: full session at HEAD (tools/round.sh: tests, smoke, PMC + SQ passes, bench, rocprof stats).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r03p bash tools/round.sh > gpurun_out/r03p_round.txt 2>&1 || { tail -30 gpurun_out/r03p_round.txt; exit 1; }
tail -14 gpurun_out/r03p_round.txt | cut -c1-600
