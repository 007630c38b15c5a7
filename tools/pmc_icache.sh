#!/bin/bash
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out; mkdir -p $OUT
for L in d1 d2; do
export PCORE_LIB=$PWD/build_ab/$L.so
i=0
for SET in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_HITS SQC_DCACHE_MISSES" "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  timeout -s KILL 90 rocprofv3 --pmc $SET --kernel-trace --output-format csv -d $OUT/ic_${L}_$i -o run -- python tools/prof_fused.py > $OUT/ic_${L}_$i.log 2>&1 || { tail -5 $OUT/ic_${L}_$i.log; exit 1; }
  i=$((i+1))
done
python - <<PY
import csv, collections
acc = collections.defaultdict(list)
for i in range(2):
    for r in csv.DictReader(open("$OUT/ic_${L}_%d/run_counter_collection.csv" % i)):
        if "fused_cost_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("== $L")
for k, v in sorted(acc.items()):
    print("%-28s %14.1f per pose" % (k, sum(v) / len(v) / 10000.0))
PY
done
