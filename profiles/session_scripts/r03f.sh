#!/bin/bash
# r03f: full measurement session at HEAD -- GICP SQ / instruction-mix passes (profiles/sq_counters_gicp.json, read by
# the bench's C3 leg), then tools/round.sh (GPU tests, smoke, PMC traffic, fused SQ counters, bench, rocprofv3 stats),
# the C1 / C3-C5 config sweep, the drop-in recognizer end to end and the C3 argmin analysis.
set -o pipefail
T=${TAG:-r03f}
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out TAG=sqg_$T bash tools/sq_gicp.sh > gpurun_out/${T}_sqg.log 2>&1 || { tail -20 gpurun_out/${T}_sqg.log; exit 1; }
python tools/sq_gicp_json.py gpurun_out sqg_$T $T > gpurun_out/${T}_sqg_json.log 2>&1 && cp profiles/sq_counters_gicp.json gpurun_out/sq_counters_gicp.json || { cat gpurun_out/${T}_sqg_json.log; exit 1; }
cat gpurun_out/${T}_sqg_json.log
TAG=$T bash tools/round.sh > gpurun_out/${T}_round.txt 2>&1 || { tail -30 gpurun_out/${T}_round.txt; exit 1; }
tail -12 gpurun_out/${T}_round.txt | cut -c1-300
timeout -k 10 600 python -u tools/bench_configs.py --configs C1,C3,C4,C5 --steps 5 > gpurun_out/${T}_configs.jsonl 2> gpurun_out/${T}_configs.err || { tail -20 gpurun_out/${T}_configs.err; exit 1; }
cut -c1-250 gpurun_out/${T}_configs.jsonl
timeout -k 10 300 python -u tools/recognizer_e2e.py > gpurun_out/${T}_e2e.txt 2>&1 || { tail -20 gpurun_out/${T}_e2e.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_e2e.txt | cut -c1-300
timeout -k 10 300 python -u tools/c3_argmin.py > gpurun_out/${T}_c3_argmin.txt 2>&1 || { tail -20 gpurun_out/${T}_c3_argmin.txt; exit 1; }
echo done
