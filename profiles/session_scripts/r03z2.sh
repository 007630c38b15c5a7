#!/bin/bash
# r03z2: final tree -- the whole GPU suite, smoke, one default bench, the drop-in end to end.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03z2_pytest.log 2>&1 || { tail -30 gpurun_out/r03z2_pytest.log; exit 1; }
tail -1 gpurun_out/r03z2_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03z2_smoke.log 2>&1 || { tail -20 gpurun_out/r03z2_smoke.log; exit 1; }
tail -1 gpurun_out/r03z2_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r03z2_bench.json 2> gpurun_out/r03z2_bench.err || { tail -20 gpurun_out/r03z2_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r03z2_bench.json')); print(round(d['value']/1e6,2), 'M poses/s', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],3), 'C3', round(d['c3']['value']/1e6,3), d['c3']['roofline']['frac_cycle_weighted'], 'cpu', round(d['cpu_baseline']['value']), round(d['cpu_reference_path']['value']))"
timeout -k 10 300 python -u tools/recognizer_e2e.py > gpurun_out/r03z2_e2e.txt 2>&1 || { tail -20 gpurun_out/r03z2_e2e.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r03z2_e2e.txt | cut -c1-160
