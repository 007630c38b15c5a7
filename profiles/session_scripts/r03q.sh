#!/bin/bash
# r03q: GICP SQ passes at HEAD (profiles/sq_counters_gicp.json for bench's C3 roofline), recognizer e2e (median).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out TAG=sqg_r03q bash tools/sq_gicp.sh > gpurun_out/r03q_sqg.log 2>&1 || { tail -20 gpurun_out/r03q_sqg.log; exit 1; }
python tools/sq_gicp_json.py gpurun_out sqg_r03q r03q > gpurun_out/r03q_sqg_json.log 2>&1 && cp profiles/sq_counters_gicp.json gpurun_out/sq_counters_gicp.json || exit 1
cat gpurun_out/r03q_sqg_json.log
timeout -k 10 300 python -u tools/recognizer_e2e.py > gpurun_out/r03q_e2e.txt 2>&1 || { tail -20 gpurun_out/r03q_e2e.txt; exit 1; }
cat gpurun_out/r03q_e2e.txt
