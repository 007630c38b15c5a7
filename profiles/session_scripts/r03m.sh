#!/bin/bash
# r03m: correspondence key with |t'|^2 added last + two-quad scan steps (key2, the working tree) vs HEAD (base):
# GICP parity of key2 (the oracle follows the new key), C3 kernel times of both (twice), key2 phase clocks.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "icp or gicp or fullsize or states or recognizer" > gpurun_out/r03m_pytest.log 2>&1 || { tail -40 gpurun_out/r03m_pytest.log; exit 1; }
tail -2 gpurun_out/r03m_pytest.log
for L in base key2 base key2; do
  PCORE_LIB=$PWD/build_ab/$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03m_$L -o run -- python tools/prof_fused.py --c3 --icp --iters 3 > gpurun_out/r03m_$L.log 2>&1 || { tail gpurun_out/r03m_$L.log; exit 1; }
  python - <<PY
import csv
for r in csv.reader(open("gpurun_out/r03m_$L/run_kernel_stats.csv")):
    if r[0] != "Name" and "gicp" in r[0]: print("$L  %-50s %8.3f ms" % (r[0][:50], float(r[3]) / 1e6))
PY
done
PCORE_LIB=$PWD/build_ab/gprof.so timeout -k 10 200 python -u tools/gicp_phase_prof.py --c3 > gpurun_out/r03m_phase.txt 2>&1
cat gpurun_out/r03m_phase.txt
timeout -k 10 300 python -u tools/recognizer_e2e.py > gpurun_out/r03m_e2e.txt 2>&1 || { tail -20 gpurun_out/r03m_e2e.txt; exit 1; }
cat gpurun_out/r03m_e2e.txt
PCORE_BENCH_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03m_c2one -o run -- python bench.py --steps 20 --no-cpu --c3-steps 0 > gpurun_out/r03m_c2one.json 2> gpurun_out/r03m_c2one.err || { tail gpurun_out/r03m_c2one.err; exit 1; }
cut -c1-200 gpurun_out/r03m_c2one.json
python - <<PY
import csv
for r in csv.reader(open("gpurun_out/r03m_c2one/run_kernel_stats.csv")):
    if r[0] != "Name" and float(r[2]) > 100000: print("  %-50s calls %s avg %8.1f us min %s max %s" % (r[0][:50], r[1], float(r[3]) / 1e3, r[5], r[6]))
PY
