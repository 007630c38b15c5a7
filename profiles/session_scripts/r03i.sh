#!/bin/bash
# r03i: GICP SQ passes at HEAD (refresh profiles/sq_counters_gicp.json), then the recognizer end-to-end timing.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out TAG=sqg_r03i bash tools/sq_gicp.sh > gpurun_out/r03i_sqg.log 2>&1 || { tail -20 gpurun_out/r03i_sqg.log; exit 1; }
python tools/sq_gicp_json.py gpurun_out sqg_r03i r03i > gpurun_out/r03i_sqg_json.log 2>&1 && cp profiles/sq_counters_gicp.json gpurun_out/sq_counters_gicp.json || exit 1
timeout -k 10 300 python -u tools/recognizer_e2e.py > gpurun_out/r03i_e2e.txt 2>&1 || { tail -20 gpurun_out/r03i_e2e.txt; exit 1; }
cat gpurun_out/r03i_e2e.txt
