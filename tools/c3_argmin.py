#!/usr/bin/env python
"""Why C3's post-GICP argmin is not always the ground-truth candidate.

Builds the C3 workload (5 objects x 10k candidates, the bench's scene), runs stage COST without and with GICP
and prints, per object: the GT candidate's integer cost before / after GICP, its GICP iterations and how far GICP
moved it (translation mm, rotation deg); the post-GICP winner's cost, iterations, pre-GICP cost and its adjusted
pose's distance to the GT pose; how many candidates end within 1 cm / 2 deg of the GT after GICP and the best
post-GICP cost among them.  Integer costs follow select_kernel (search_env.cpp:1987-2051); -1 = filtered."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from perception_amd import workloads  # noqa: E402

NAMES = ["003_cracker_box", "005_tomato_soup_can", "006_mustard_bottle", "010_potted_meat_can", "024_bowl"]


def int_costs(rc, oc):
    """select_kernel's integer cost, -1 where the reference's filter drops the pose."""
    rc = rc.astype(np.float32)
    oc = oc.astype(np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        t = np.where(np.isfinite(rc), rc, 0).astype(np.int64)
        s = np.where(np.isfinite(oc), oc, 0).astype(np.int64)
        c = np.where(t < 0, -1, (rc + oc).astype(np.float32).astype(np.int64))
    c[np.abs(t - s) >= 30] = -1
    return c


def rel(a, b):
    """Translation (mm) and rotation (deg) between two cm-scaled mat4x4 rows (init_from_eigen layout)."""
    A = a.reshape(4, 4).astype(np.float64) / 100.0  # init_from_eigen scales rows 0-2 (rotation too) by 100
    B = b.reshape(4, 4).astype(np.float64) / 100.0
    dt = np.linalg.norm(A[:3, 3] - B[:3, 3]) * 1000.0  # m -> mm
    R = A[:3, :3] @ B[:3, :3].T
    ang = np.degrees(np.arccos(np.clip((np.trace(R) - 1) / 2, -1, 1)))
    return round(float(dt), 2), round(float(ang), 3)


def main():
    w = workloads.build(names=NAMES, poses_per_model=10000)
    rc0, oc0, _ = w.core.evaluate(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=w.stride)
    adj, its, rc1, oc1, _ = w.core.evaluate_icp(w.poses, w.pose_model, w.pose_label, w.pose_obs_total,
                                                stride=w.stride)
    torch.cuda.synchronize()
    P = w.poses.cpu().numpy()
    A = adj.cpu().numpy()
    it = its.cpu().numpy()
    pm = w.pose_model.cpu().numpy()
    c0 = int_costs(rc0.cpu().numpy(), oc0.cpu().numpy())
    c1 = int_costs(rc1.cpu().numpy(), oc1.cpu().numpy())
    out = []
    for m, g in enumerate(w.gt_index):
        idx = np.nonzero(pm == m)[0]
        ok = idx[c1[idx] >= 0]
        win = int(ok[np.argmin(c1[ok])]) if len(ok) else -1  # first minimum = lowest index
        gt_pose = P[g]
        def close(i):
            dt, ang = rel(A[i], gt_pose)
            return dt < 10.0 and ang < 2.0
        near = [i for i in ok if close(i)]
        best_near = min((int(c1[i]) for i in near), default=None)
        r = {"object": NAMES[m], "gt_index": int(g), "gt_cost_before": int(c0[g]), "gt_cost_after": int(c1[g]),
             "gt_iters": int(it[g]), "gt_moved_mm_deg": rel(A[g], gt_pose),
             "winner": win, "winner_cost_after": int(c1[win]), "winner_cost_before": int(c0[win]),
             "winner_iters": int(it[win]), "winner_to_gt_mm_deg": rel(A[win], gt_pose),
             "winner_start_to_gt_mm_deg": rel(P[win], gt_pose),
             "within_1cm_2deg_after": len(near), "best_cost_within_1cm_2deg": best_near,
             "cost_after_hist": {str(k): int(v) for k, v in zip(*np.unique(np.clip(c1[ok], -1, 60), return_counts=True))
                                 if k <= 10}}
        # the GT candidate's rendered / observed cost parts before and after, and stage COST (no ICP) of its
        # adjusted pose: the post-GICP re-score must equal it
        sel = torch.tensor([g, win], dtype=torch.long, device=w.poses.device)
        rcA, ocA, _ = w.core.evaluate(adj[sel].contiguous(), w.pose_model[sel].contiguous(),
                                      w.pose_label[sel].contiguous(), w.pose_obs_total[sel].contiguous(),
                                      stride=w.stride)
        r["gt_rc_oc_before"] = [float(rc0[g]), float(oc0[g])]
        r["gt_rc_oc_after"] = [float(rc1[g]), float(oc1[g])]
        r["gt_rc_oc_rescored"] = [float(rcA[0]), float(ocA[0])]
        r["winner_rc_oc_after"] = [float(rc1[win]), float(oc1[win])]
        r["gt_adjusted_minus_start"] = np.round(A[g] - P[g], 5).tolist()
        # the GT pose moved by GICP's translation only (rotation kept): isolates the translation's effect
        shifted = P[g].copy()
        shifted[[3, 7, 11]] = A[g][[3, 7, 11]]
        rcS, ocS, _ = w.core.evaluate(torch.from_numpy(shifted[None]).to(w.poses.device), w.pose_model[g:g + 1],
                                      w.pose_label[g:g + 1], w.pose_obs_total[g:g + 1], stride=w.stride)
        r["gt_translated_only_rc_oc"] = [float(rcS[0]), float(ocS[0])]
        out.append(r)
        print(json.dumps(r), flush=True)
    return out


if __name__ == "__main__":
    main()
