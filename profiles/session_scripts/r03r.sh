#!/bin/bash
# r03r: GICP SQ passes at HEAD (profiles/sq_counters_gicp.json), recognizer e2e (median), C3 argmin analysis,
# LDS bank-conflict A/B of the conditional fragment atomic (build_ab/base.so vs build_ab/atomif.so).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out TAG=sqg_r03r bash tools/sq_gicp.sh > gpurun_out/r03r_sqg.log 2>&1 || { tail -20 gpurun_out/r03r_sqg.log; exit 1; }
python tools/sq_gicp_json.py gpurun_out sqg_r03r r03r > gpurun_out/r03r_sqg_json.log 2>&1 && cp profiles/sq_counters_gicp.json gpurun_out/sq_counters_gicp.json || exit 1
cat gpurun_out/r03r_sqg_json.log
timeout -k 10 300 python -u tools/recognizer_e2e.py > gpurun_out/r03r_e2e.txt 2>&1 || { tail -20 gpurun_out/r03r_e2e.txt; exit 1; }
cat gpurun_out/r03r_e2e.txt
timeout -k 10 300 python -u tools/c3_argmin.py > gpurun_out/r03r_c3_argmin.txt 2>&1 || { tail -20 gpurun_out/r03r_c3_argmin.txt; exit 1; }
cat gpurun_out/r03r_c3_argmin.txt
PCORE_LIB=$PWD/build_ab/atomif.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fused or render or random or window" > gpurun_out/r03r_pytest_atomif.log 2>&1 || { tail -30 gpurun_out/r03r_pytest_atomif.log; exit 1; }
tail -1 gpurun_out/r03r_pytest_atomif.log
LIBS="build_ab/base.so build_ab/atomif.so" MASKS="0 1" bash tools/lds_conflicts.sh > gpurun_out/r03r_lds.txt 2>&1 || { tail -20 gpurun_out/r03r_lds.txt; exit 1; }
cat gpurun_out/r03r_lds.txt
LIBS="build_ab/base.so build_ab/atomif.so build_ab/base.so build_ab/atomif.so" CONFIGS=C2 bash tools/lib_ab.sh > gpurun_out/r03r_ab.txt 2>&1 || { tail -20 gpurun_out/r03r_ab.txt; exit 1; }
cat gpurun_out/r03r_ab.txt
