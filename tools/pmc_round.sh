#!/bin/bash
# HBM traffic of the fused kernel from PMC counters: separate passes for FETCH_SIZE and WRITE_SIZE
# (MI355X_MICROARCH.md "HBM": never combine --pmc with trace domains).
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-r01}
export TMPDIR=/tmp
mkdir -p $OUT
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_${TAG}_$C -o run -- python bench.py --steps 3 --warmup 1 --no-cpu > $OUT/pmc_${TAG}_$C.json 2> $OUT/pmc_${TAG}_$C.err || { tail -20 $OUT/pmc_${TAG}_$C.err; exit 1; }
done
find $OUT -path "*pmc_${TAG}*" -name "*.csv" | head
