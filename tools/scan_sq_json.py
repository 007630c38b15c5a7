#!/usr/bin/env python
"""Fold tools/scan_sq.sh's counter passes: per mesh, the fused kernel's SQ_INSTS_VALU / SALU / LDS per pose of the
10,000-pose launches, beside the mesh's triangles and the stream builder's vertex passes and steps (the per-element
costs of DESIGN.md section 4).  Usage: scan_sq_json.py OUT_DIR"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out):
    from perception_amd import synthetic as syn
    from tools.step_skip_estimate import stream_steps

    res = {}
    for p in sorted(glob.glob(os.path.join(out, "sq_*", "*counter_collection.csv"))):
        mesh = os.path.basename(os.path.dirname(p))[3:]
        vals = {}
        for r in csv.DictReader(open(p)):
            if "fused_cost_kernel" in r["Kernel_Name"] and int(r["Grid_Size"]) == 10000 * 256:
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        if not vals:
            continue
        v = {k: sum(x) / len(x) for k, x in vals.items()}
        tris = syn.ycb_proxy(mesh).tris
        steps = stream_steps(tris)
        res[mesh] = {"triangles": int(len(tris)), "stream_steps": int(len(steps)),
                     "valu_per_pose": v["SQ_INSTS_VALU"] / 10000, "salu_per_pose": v.get("SQ_INSTS_SALU", 0) / 10000,
                     "lds_per_pose": v.get("SQ_INSTS_LDS", 0) / 10000,
                     "valu_per_triangle": v["SQ_INSTS_VALU"] / 10000 / len(tris),
                     "launches": len(vals["SQ_INSTS_VALU"])}
    s = json.dumps(res, indent=1)
    print(s)
    with open(os.path.join(out, "scan_valu.json"), "w") as f:
        f.write(s + "\n")


if __name__ == "__main__":
    main(sys.argv[1])
