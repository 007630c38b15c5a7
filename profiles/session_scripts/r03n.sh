#!/bin/bash
# r03n: recognizer end-to-end with the state-generation split; C2 workgroup timeline (per-pose durations, for the
# launch-order study of the single-stream drain).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/recognizer_e2e.py > gpurun_out/r03n_e2e.txt 2>&1 || { tail -20 gpurun_out/r03n_e2e.txt; exit 1; }
cat gpurun_out/r03n_e2e.txt
PCORE_BENCH_LANES=1 PCORE_LIB=$PWD/build_ab/wgt.so timeout -k 10 300 python -u tools/wg_timeline.py --dump gpurun_out/r03n_wgt.npz > gpurun_out/r03n_wgt.txt 2>&1 || { tail -20 gpurun_out/r03n_wgt.txt; exit 1; }
cat gpurun_out/r03n_wgt.txt
