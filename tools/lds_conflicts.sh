#!/bin/bash
# LDS bank conflicts of the fused kernel per library build (LIBS) and PCORE_DEBUG_SKIP ablation mask (MASKS: 1 skips
# the record flush, 2 the triangle stage, 4 phase 2, 8 the vertex stage): SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE of
# one counters-only rocprofv3 pass each, on the C2 launch of tools/prof_fused.py.  Masks other than 0 need builds with
# -DPCORE_DEBUG_SKIP_RT=1 (tools/build_variant.sh NAME -DPCORE_DEBUG_SKIP_RT=1): the production library ignores them.
set -o pipefail
OUT=${OUT:-gpurun_out}; export TMPDIR=/tmp; mkdir -p $OUT
for L in ${LIBS:-perception_amd/libpcore.so}; do
  T=$(basename $L .so); export PCORE_LIB=$PWD/$L
  for M in ${MASKS:-0}; do
    PCORE_DEBUG_SKIP=$M timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/ldsc_${T}_$M -o run -- python tools/prof_fused.py > $OUT/ldsc_${T}_$M.log 2>&1 || { tail -5 $OUT/ldsc_${T}_$M.log; exit 1; }
    python - <<PY
import csv, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open("$OUT/ldsc_${T}_$M/run_counter_collection.csv")):
    if "fused_cost_kernel" in r["Kernel_Name"] and int(r["Grid_Size"]) == 10000 * 256:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in acc.items()}
print("$T skip=$M conflict/idx_active %.3f  conflict %.2fM  idx_active %.2fM  lds_instr/pose %.0f  valu/pose %.0f  gui %.0f" % (
    m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"], m["SQ_LDS_BANK_CONFLICT"] / 1e6, m["SQ_LDS_IDX_ACTIVE"] / 1e6,
    m["SQ_INSTS_LDS"] / 1e4, m["SQ_INSTS_VALU"] / 1e4, m["GRBM_GUI_ACTIVE"]))
PY
  done
done
