#!/bin/bash
# SQ_INSTS_VALU per pose of the fused kernel on C2's single-mesh workload for the box proxy and the two scan-like
# irregular meshes (one counters-only rocprofv3 pass each), folded by tools/scan_sq_json.py.  TAG names the outputs.
set -o pipefail
OUT=gpurun_out/${TAG:-ssq}; mkdir -p $OUT; export TMPDIR=/tmp
for M in 003_cracker_box scan_blob scan_shell; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
    -d $OUT/sq_$M -o run -- python tools/prof_fused.py --mesh $M > $OUT/sq_$M.log 2>&1 || { tail -20 $OUT/sq_$M.log; exit 1; }
done
python tools/scan_sq_json.py $OUT
