#!/bin/bash
# SQ counters of covariance_kernel on C3 (the source covariances of one evaluate_icp call): two counters-only passes,
# folded by tools/cov_sq_json.py.  TAG names the outputs.
set -o pipefail
OUT=gpurun_out/${TAG:-csq}; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  timeout -s KILL 180 rocprofv3 --pmc $SET --kernel-trace --output-format csv -d $OUT/cov_$i -o run -- python tools/prof_fused.py --c3 --icp --iters 1 > $OUT/cov_$i.log 2>&1 || { tail -20 $OUT/cov_$i.log; exit 1; }
  i=$((i+1))
done
python - "$OUT" <<'PY'
import csv, glob, json, os, sys
KPAT = os.environ.get("KPAT", "covariance_cloud_kernel")
out = sys.argv[1]
v = {}
for p in sorted(glob.glob(out + "/cov_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(p)):
        if KPAT in r["Kernel_Name"] and int(r["Grid_Size"]) >= 64 * 40000:
            v.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
m = {k: sum(x) / len(x) for k, x in v.items()}
if "SQ_INSTS_VALU" in m and "GRBM_GUI_ACTIVE" in m:
    m["valu_issue_frac_at_2cyc"] = 2 * m["SQ_INSTS_VALU"] / (1024 * m["GRBM_GUI_ACTIVE"] / 8)
if "SQ_WAIT_INST_ANY" in m:
    m["wait_inst_any_frac"] = m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"]
    m["active_valu_frac"] = m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"]
print(json.dumps(m, indent=1))
json.dump(m, open(out + "/cov_sq.json", "w"), indent=1)
PY
