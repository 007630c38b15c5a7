#!/bin/bash
# Same-box A/B of environment settings on bench.py's C3 leg (and the C2 line):
#   RUNS="nohist:PCORE_GICP_NO_HIST=1 hist:" REPS=2 tools/c3_env_ab.sh
set -o pipefail
OUT=${OUT:-gpurun_out}; export TMPDIR=/tmp; mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for r in $RUNS; do
    N=${r%%:*}; E=${r#*:}; E=${E//,/ }
    env $E timeout -k 10 300 python bench.py --no-cpu --steps ${C2_STEPS:-5} --c3-steps ${C3_STEPS:-5} > $OUT/c3envab_$N.json 2> $OUT/c3envab_$N.err || { tail -20 $OUT/c3envab_$N.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/c3envab_$N.json')); c=d['c3']; g=c['gicp']; print('$N: C2 %.4gM  C3 %.4gM poses/s  %.2f ms/step  gicp %.3f ms  it %.1f' % (d['value']/1e6, c['value']/1e6, c['ms_per_step'], g['gicp_ms_per_step'], g['iterations_mean']))"
  done
done
