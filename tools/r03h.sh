#!/bin/bash
# r03h: full measurement session at HEAD - tests/smoke/PMC/SQ/bench/rocprof (tools/round.sh), then the GICP SQ
# passes (refresh profiles/sq_counters_gicp.json), the C3 per-config line and the recognizer end-to-end timing.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r03h bash tools/round.sh > gpurun_out/r03h_round.txt 2>&1 || { tail -30 gpurun_out/r03h_round.txt; exit 1; }
OUT=gpurun_out TAG=sqg_r03h bash tools/sq_gicp.sh > gpurun_out/r03h_sqg.log 2>&1 || { tail -20 gpurun_out/r03h_sqg.log; exit 1; }
python tools/sq_gicp_json.py gpurun_out sqg_r03h r03h > gpurun_out/r03h_sqg_json.log 2>&1 && cp profiles/sq_counters_gicp.json gpurun_out/sq_counters_gicp.json || exit 1
timeout -k 10 300 python -u tools/recognizer_e2e.py > gpurun_out/r03h_e2e.txt 2>&1 || { tail -20 gpurun_out/r03h_e2e.txt; exit 1; }
tail -3 gpurun_out/r03h_round.txt; cat gpurun_out/r03h_e2e.txt
