#!/bin/bash
# SQ instruction-mix counters of the fused kernel (two counters-only passes): which VALU kinds (transcendental,
# 64-bit, conversions, f32 fma / mul / add, int32) and how much scalar / branch / LDS work one pose issues.
set -o pipefail
OUT=${OUT:-gpurun_out}; TAG=${TAG:-mix}
export TMPDIR=/tmp
mkdir -p $OUT
i=0
for SET in "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32" \
           "SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_VSKIPPED GRBM_GUI_ACTIVE"; do
  timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-trace --output-format csv -d $OUT/${TAG}_$i -o run -- python tools/prof_fused.py ${ARGS} > $OUT/${TAG}_$i.log 2>&1 || { tail -20 $OUT/${TAG}_$i.log; exit 1; }
  i=$((i+1))
done
python - <<PY
import csv, collections
acc = collections.defaultdict(list)
for i in range(2):
    for r in csv.DictReader(open("$OUT/${TAG}_%d/run_counter_collection.csv" % i)):
        if "fused_cost_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    # one row per dispatch per counter (summed over dimensions by rocprofv3); report the per-dispatch mean / 10k poses
    print("%-26s %12.1f per pose" % (k, sum(v) / len(v) / 10000.0))
PY
