#!/bin/bash
# r03f: full measurement session at HEAD -- GICP SQ / instruction-mix passes (profiles/sq_counters_gicp.json, read by
# the bench's C3 leg), then tools/round.sh (GPU tests, smoke, PMC traffic, fused SQ counters, bench, rocprofv3 stats),
# the C1 / C3-C5 config sweep, the drop-in recognizer end to end and the C3 argmin analysis.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out TAG=sqg_r03f bash tools/sq_gicp.sh > gpurun_out/r03f_sqg.log 2>&1 || { tail -20 gpurun_out/r03f_sqg.log; exit 1; }
python tools/sq_gicp_json.py gpurun_out sqg_r03f r03f > gpurun_out/r03f_sqg_json.log 2>&1 && cp profiles/sq_counters_gicp.json gpurun_out/sq_counters_gicp.json || { cat gpurun_out/r03f_sqg_json.log; exit 1; }
cat gpurun_out/r03f_sqg_json.log
TAG=r03f bash tools/round.sh > gpurun_out/r03f_round.txt 2>&1 || { tail -30 gpurun_out/r03f_round.txt; exit 1; }
tail -12 gpurun_out/r03f_round.txt | cut -c1-300
timeout -k 10 600 python -u tools/bench_configs.py --configs C1,C3,C4,C5 --steps 5 > gpurun_out/r03f_configs.jsonl 2> gpurun_out/r03f_configs.err || { tail -20 gpurun_out/r03f_configs.err; exit 1; }
cut -c1-250 gpurun_out/r03f_configs.jsonl
timeout -k 10 300 python -u tools/recognizer_e2e.py > gpurun_out/r03f_e2e.txt 2>&1 || { tail -20 gpurun_out/r03f_e2e.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r03f_e2e.txt | cut -c1-300
timeout -k 10 300 python -u tools/c3_argmin.py > gpurun_out/r03f_c3_argmin.txt 2>&1 || { tail -20 gpurun_out/r03f_c3_argmin.txt; exit 1; }
echo done
