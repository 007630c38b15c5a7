#!/bin/bash
# r03l: four poses per wave (gicp_group_kernel): GICP parity tests, C3 kernel stats + throughput, phase clocks.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "icp or gicp or fullsize or recognizer or distributed" > gpurun_out/r03l_pytest.log 2>&1 || { tail -40 gpurun_out/r03l_pytest.log; exit 1; }
tail -3 gpurun_out/r03l_pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03l_c3prof -o run -- python tools/prof_fused.py --c3 --icp --iters 3 > gpurun_out/r03l_c3prof.log 2>&1 || { tail gpurun_out/r03l_c3prof.log; exit 1; }
python - <<PY
import csv
for r in csv.reader(open("gpurun_out/r03l_c3prof/run_kernel_stats.csv")):
    if r[0] != "Name" and float(r[3]) > 100000: print("  %-50s %8.3f ms" % (r[0][:50], float(r[3]) / 1e6))
PY
timeout -k 10 300 python tools/bench_configs.py --configs C3 --steps 5 > gpurun_out/r03l_c3.jsonl 2> gpurun_out/r03l_c3.err || { tail gpurun_out/r03l_c3.err; exit 1; }
cut -c1-400 gpurun_out/r03l_c3.jsonl
PCORE_LIB=$PWD/build_ab/gprof.so timeout -k 10 200 python -u tools/gicp_phase_prof.py --c3 > gpurun_out/r03l_phase.txt 2>&1
cat gpurun_out/r03l_phase.txt
