#!/bin/bash
# r03h: full measurement session at HEAD - tests/smoke/PMC/SQ/bench/rocprof (tools/round.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r03h bash tools/round.sh > gpurun_out/r03h_round.txt 2>&1 || { tail -30 gpurun_out/r03h_round.txt; exit 1; }
tail -12 gpurun_out/r03h_round.txt
