#!/bin/bash
# r03o: fused argmin (pcore_evaluate_select): parity tests, one-lane and two-lane C2 bench, recognizer e2e.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "select or recognizer or tabletop or states or sweep or distributed" > gpurun_out/r03o_pytest.log 2>&1 || { tail -40 gpurun_out/r03o_pytest.log; exit 1; }
tail -2 gpurun_out/r03o_pytest.log
for L in 1 2 1 2; do
  PCORE_BENCH_LANES=$L timeout -k 10 300 python bench.py --steps 40 --no-cpu --c3-steps 0 > gpurun_out/r03o_c2_lanes$L.json 2> gpurun_out/r03o_c2.err || { tail gpurun_out/r03o_c2.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r03o_c2_lanes$L.json')); print('lanes $L', round(d['value']/1e6,3), 'M poses/s', round(d['ms_per_step'],4), 'ms')"
done
timeout -k 10 300 python -u tools/recognizer_e2e.py > gpurun_out/r03o_e2e.txt 2>&1 || { tail -20 gpurun_out/r03o_e2e.txt; exit 1; }
cat gpurun_out/r03o_e2e.txt
