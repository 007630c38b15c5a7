#!/usr/bin/env python
"""Fold the counter passes of tools/sq_counters.sh into profiles/sq_counters.json (the fused_cost entry:
per-counter mean over the batch-size launches of fused_cost_kernel, the VALU instructions per pose and the
issue rate, tagged with the digest of the kernel sources it measured; bench.py reports roofline from it and
refuses a profile of other sources).  Usage: sq_json.py OUT_DIR TAG [poses_per_launch] [round]"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from perception_amd.build import kernel_source_digest  # noqa: E402


def main(out_dir, tag, poses=10000, rnd=None):
    poses = int(poses)
    vals = defaultdict(list)
    meta = {}
    for p in sorted(glob.glob(os.path.join(out_dir, f"{tag}_*", "*counter_collection.csv"))):
        rows = [r for r in csv.DictReader(open(p)) if "fused_cost_kernel" in r["Kernel_Name"]
                and int(r["Grid_Size"]) == poses * 256]
        for r in rows:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = {"_grid": float(r["Grid_Size"]), "_lds": float(r["LDS_Block_Size"]),
                    "_sgpr": float(r["SGPR_Count"]), "_vgpr": float(r["VGPR_Count"])}
    if "SQ_INSTS_VALU" not in vals or "GRBM_GUI_ACTIVE" not in vals:
        sys.exit("no fused_cost_kernel SQ_INSTS_VALU / GRBM_GUI_ACTIVE rows found")
    fc = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
    fc.update(meta)
    per_simd_cycle = fc["SQ_INSTS_VALU"] / (1024.0 * fc["GRBM_GUI_ACTIVE"] / 8.0)
    fc["derived_valu_instr_per_simd_cycle"] = per_simd_cycle
    fc["derived_valu_issue_frac_at_2cyc"] = 2.0 * per_simd_cycle
    fc["derived_valu_instr_per_pose"] = fc["SQ_INSTS_VALU"] / poses
    if "SQ_INSTS_SALU" in fc:
        fc["derived_salu_instr_per_pose"] = fc["SQ_INSTS_SALU"] / poses
    if "SQ_INSTS_LDS" in fc:
        fc["derived_lds_instr_per_pose"] = fc["SQ_INSTS_LDS"] / poses
    path = os.path.join(ROOT, "profiles", "sq_counters.json")
    d = json.load(open(path)) if os.path.exists(path) else {}
    d["fused_cost"] = fc
    d["fused_cost_poses_per_launch"] = poses
    d["kernel_source_digest"] = kernel_source_digest()
    d["note"] = ("tools/sq_counters.sh passes (counters only); fused_cost = C2 10k-pose launch; GRBM_GUI_ACTIVE "
                 "summed over 8 XCDs; issue fraction assumes 2 cycles per wave64 VALU instruction "
                 "(MI355X_MICROARCH.md)")
    json.dump(d, open(path, "w"), indent=1)
    if rnd:
        shutil.copy(path, os.path.join(ROOT, "profiles", f"{rnd}_sq_counters.json"))
    print(json.dumps({k: v for k, v in fc.items() if k.startswith("derived")}))


if __name__ == "__main__":
    main(*sys.argv[1:])
