#!/bin/bash
# Instruction counts of the fused kernel under PCORE_DEBUG_SKIP ablations (one counters-only rocprofv3 pass
# per mask): what the flush (1), the triangle stage (2), phase 2 (4) and the vertex stage (8) each issue.
set -o pipefail
OUT=${OUT:-gpurun_out}; export TMPDIR=/tmp; mkdir -p $OUT
# the production build ignores PCORE_DEBUG_SKIP: these passes load an ablation build
# (tools/build_variant.sh ablate -DPCORE_DEBUG_SKIP_RT=1, made here on the CPU beforehand)
export PCORE_LIB=${PCORE_LIB:-$PWD/build_ab/ablate.so}
[ -f "$PCORE_LIB" ] || { echo "missing $PCORE_LIB (tools/build_variant.sh ablate -DPCORE_DEBUG_SKIP_RT=1)"; exit 1; }
for M in ${MASKS:-0 1 2 4 8 15}; do
  PCORE_DEBUG_SKIP=$M timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/absq_$M -o run -- python tools/prof_fused.py > $OUT/absq_$M.log 2>&1 || { tail -5 $OUT/absq_$M.log; exit 1; }
done
python - <<PY
import csv, collections
for m in "${MASKS:-0 1 2 4 8 15}".split():
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open("$OUT/absq_%s/run_counter_collection.csv" % m)):
        if "fused_cost_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("skip=%-3s " % m + "  ".join("%s %.0f" % (k.replace("SQ_", ""), sum(v) / len(v) / 1e4) for k, v in sorted(acc.items())))
PY
