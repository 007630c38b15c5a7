#!/usr/bin/env python
"""Fold the counter passes of tools/sq_gicp.sh into profiles/sq_counters_gicp.json: per-counter values of the
gicp_kernel launch of the profiled C3 call, the VALU instructions per pose-iteration (the launch's SQ_INSTS_VALU
over the call's summed GICP iterations) and the issue fraction, tagged with the digest of the GICP sources (bench.py
refuses a profile of other sources).  Usage: sq_gicp_json.py OUT_DIR TAG [round]"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from perception_amd.build import gicp_source_digest  # noqa: E402


def main(out_dir, tag, rnd=None):
    it = json.load(open(os.path.join(out_dir, f"{tag}_iters.json")))
    vals = defaultdict(list)
    meta = {}
    for p in sorted(glob.glob(os.path.join(out_dir, f"{tag}_*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"]
            if "gicp_kernel" not in name or "wide" in name or "cost_key" in name:
                continue
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = {"_grid": float(r["Grid_Size"]), "_lds": float(r["LDS_Block_Size"]),
                    "_sgpr": float(r["SGPR_Count"]), "_vgpr": float(r["VGPR_Count"])}
    if "SQ_INSTS_VALU" not in vals or "GRBM_GUI_ACTIVE" not in vals:
        sys.exit("no gicp_kernel SQ_INSTS_VALU / GRBM_GUI_ACTIVE rows found")
    gk = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
    gk.update(meta)
    pi = it["pose_iterations"]
    per_simd_cycle = gk["SQ_INSTS_VALU"] / (1024.0 * gk["GRBM_GUI_ACTIVE"] / 8.0)
    gk["derived_valu_instr_per_simd_cycle"] = per_simd_cycle
    gk["derived_valu_issue_frac_at_2cyc"] = 2.0 * per_simd_cycle
    gk["derived_valu_instr_per_pose_iteration"] = gk["SQ_INSTS_VALU"] / pi
    for c in ("SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD"):
        if c in gk:
            gk["derived_" + c[9:].lower() + "_per_pose_iteration"] = gk[c] / pi
    if "SQ_WAIT_INST_ANY" in gk and "SQ_WAVE_CYCLES" in gk:
        gk["derived_wait_inst_any_frac"] = gk["SQ_WAIT_INST_ANY"] / gk["SQ_WAVE_CYCLES"]
    f64 = sum(gk.get(c, 0.0) for c in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64"))
    trans = gk.get("SQ_INSTS_VALU_TRANS_F64", 0.0) + gk.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
    if "SQ_INSTS_VALU_FMA_F64" in gk:
        # SIMD cycles the VALU work occupies: f64 FMA / MUL / ADD and transcendentals 4 cycles per wave64
        # instruction (tools/exec_half.hip: v_fma_f64 4.15 cycles at full occupancy; MI355X_MICROARCH.md: the
        # transcendentals twice an FMA's issue cost), every other VALU instruction 2
        cyc = 2.0 * (gk["SQ_INSTS_VALU"] - f64 - trans) + 4.0 * (f64 + trans)
        gk["derived_f64_frac_of_valu"] = f64 / gk["SQ_INSTS_VALU"]
        gk["derived_valu_cycles_per_pose_iteration"] = cyc / pi
        gk["derived_valu_busy_frac_cycle_weighted"] = cyc / (1024.0 * gk["GRBM_GUI_ACTIVE"] / 8.0)
    if "SQ_LDS_BANK_CONFLICT" in gk and "SQ_LDS_IDX_ACTIVE" in gk:
        gk["derived_lds_bank_conflict_frac"] = gk["SQ_LDS_BANK_CONFLICT"] / max(gk["SQ_LDS_IDX_ACTIVE"], 1.0)
    d = {"gicp_kernel": gk, "poses": it["poses"], "pose_iterations": pi, "gicp_source_digest": gicp_source_digest(),
         "note": "tools/sq_gicp.sh passes (counters only) over one C3 evaluate_icp (50k poses, one chunk); "
                 "GRBM_GUI_ACTIVE summed over 8 XCDs; issue fraction assumes 2 cycles per wave64 VALU instruction "
                 "(MI355X_MICROARCH.md)"}
    path = os.path.join(ROOT, "profiles", "sq_counters_gicp.json")
    json.dump(d, open(path, "w"), indent=1)
    if rnd:
        shutil.copy(path, os.path.join(ROOT, "profiles", f"{rnd}_sq_counters_gicp.json"))
    print(json.dumps({k: v for k, v in gk.items() if k.startswith("derived")}))


if __name__ == "__main__":
    main(*sys.argv[1:])
