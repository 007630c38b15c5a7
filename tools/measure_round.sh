#!/bin/bash
# Measurement session (no parity tests): headline bench, rocprofv3 stats of the bench, the other
# BASELINE configs (C3 with GICP + ADD-S), GICP phase clocks.  Each GPU step has its own time limit.
set -o pipefail
OUT=${OUT:-gpurun_out}; TAG=${TAG:-m}
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps ${STEPS:-20} --warmup 3 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python bench.py --steps 10 --warmup 2 --no-cpu > $OUT/prof_bench_$TAG.json 2> $OUT/prof_$TAG.err || { tail -20 $OUT/prof_$TAG.err; exit 1; }
timeout -k 10 900 python tools/bench_configs.py --configs ${CONFIGS:-C2,C3,C4,C5} --steps 3 > $OUT/configs_$TAG.jsonl 2> $OUT/configs_$TAG.err || { tail -20 $OUT/configs_$TAG.err; exit 1; }
cat $OUT/configs_$TAG.jsonl | cut -c1-400
if [ -f build_ab/prof.so ]; then
  PCORE_LIB=$PWD/build_ab/prof.so timeout -k 10 300 python tools/gicp_phase_prof.py > $OUT/gicp_phase_$TAG.log 2>&1 || { tail $OUT/gicp_phase_$TAG.log; exit 1; }
  cat $OUT/gicp_phase_$TAG.log
fi
