#!/bin/bash
# Round 6 GPU checks beside GICP: the one-rank RCCL exchange (lane pattern), the scan-mesh parity tests and the scan
# meshes' C2 / C3 configs.  Each step under its own time limit; the chain stops at the first failure.
set -o pipefail
OUT=gpurun_out/${TAG:-mc}
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/rccl_lane_check.py --steps 12 --poses 2000 > $OUT/rccl_lane_check.json 2> $OUT/rccl_lane_check.err \
  || { tail -30 $OUT/rccl_lane_check.err; exit 1; }
cat $OUT/rccl_lane_check.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTS:-scan or rccl or distributed}" \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 python -u bench.py --no-cpu --force-pg --c3-steps 0 > $OUT/bench_force_pg.json 2> $OUT/bench_force_pg.err || { tail -20 $OUT/bench_force_pg.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_force_pg.json')); print('force-pg C2 %.4g M poses/s' % (d['value']/1e6), d['config']['dist_backend'], d['config']['exchange'], d['host_timing']['exchange_issue_ms'])"
timeout -k 10 400 python -u bench.py --no-cpu --c3-steps 0 > $OUT/bench_no_pg.json 2> $OUT/bench_no_pg.err || { tail -20 $OUT/bench_no_pg.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_no_pg.json')); print('no-pg C2 %.4g M poses/s' % (d['value']/1e6), d['config']['dist_backend'])"
timeout -k 10 600 python -u tools/bench_configs.py --configs C2,C2scan_blob,C2scan_shell,C3scan > $OUT/configs_scan.jsonl 2> $OUT/configs_scan.err || { tail -20 $OUT/configs_scan.err; exit 1; }
python -c "
import json
for l in open('$OUT/configs_scan.jsonl'):
    d = json.loads(l); print(d['config'], d['triangles'], '%.4g M poses/s' % (d['poses_per_s'] / 1e6), 'adds_auc', d['adds_auc'])"
