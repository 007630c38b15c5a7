#!/bin/bash
# r03t: C3 argmin analysis (rotation normalised) and the C1-C5 config sweep at HEAD.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/c3_argmin.py > gpurun_out/r03t_c3_argmin.txt 2>&1 || { tail -20 gpurun_out/r03t_c3_argmin.txt; exit 1; }
cat gpurun_out/r03t_c3_argmin.txt
timeout -k 10 600 python -u tools/bench_configs.py --configs C1,C3,C4,C5 --steps 5 > gpurun_out/r03t_configs.jsonl 2> gpurun_out/r03t_configs.err || { tail -20 gpurun_out/r03t_configs.err; exit 1; }
cut -c1-400 gpurun_out/r03t_configs.jsonl
