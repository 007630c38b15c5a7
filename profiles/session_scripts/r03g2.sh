#!/bin/bash
# r03g2: final-tree check -- the whole GPU suite, smoke, and three back-to-back default bench runs (run-to-run spread).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03g2_pytest.log 2>&1 || { tail -30 gpurun_out/r03g2_pytest.log; exit 1; }
tail -1 gpurun_out/r03g2_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03g2_smoke.log 2>&1 || { tail -20 gpurun_out/r03g2_smoke.log; exit 1; }
tail -1 gpurun_out/r03g2_smoke.log
for i in 1 2 3; do
  timeout -k 10 600 python bench.py > gpurun_out/r03g2_bench$i.json 2> gpurun_out/r03g2_bench$i.err || { tail -20 gpurun_out/r03g2_bench$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r03g2_bench$i.json')); print(round(d['value']/1e6,2), 'M poses/s', round(d['ms_per_step'],4), 'ms/step frac', round(d['roofline']['frac'],3), 'C3', round(d['c3']['value']/1e6,3), 'M', round(d['c3']['ms_per_step'],2), 'ms', d['c3']['roofline']['frac_cycle_weighted'])"
done
