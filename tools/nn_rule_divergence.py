#!/usr/bin/env python
"""How far the spec's correspondence rule (the centred FMA key |q'-t'|^2 - |q'|^2, pcore_gicp_math.h nn_key; first
strict minimum) leads GICP away from the exact float32 squared-distance rule that fast_gicp's brute-force k = 1 search
ranks by.  CPU only:
  * per query: over every linearisation of every candidate's oracle trace, how often the two rules pick a different
    target, and the float squared distance the key rule gives up when they do;
  * per pose: the oracle's GICP (key rule, bit-exact with the kernels) against tests/gicp_reference.py's numpy chain
    with its own exact-distance search -- iteration counts and the transform difference.
    python tools/nn_rule_divergence.py [--poses-per-object 24] [--seed 7] [--c1] [--out FILE.json]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from tests import gicp_reference as gref  # noqa: E402
from tests.helpers import SceneCase  # noqa: E402

C3_NAMES = ("003_cracker_box", "004_sugar_box", "005_tomato_soup_can", "006_mustard_bottle", "010_potted_meat_can")


def c3_pairs(n, seed):
    case = SceneCase(names=C3_NAMES, n_poses=n, seed=seed)
    sc = case.scene
    depth = oracle.render_depth(sc.bank.tris, sc.bank.tris_model_count, case.poses, case.pose_model, case.pose_label,
                                sc.width, sc.height, sc.proj, sc.src_depth_cm, sc.mask, 1.0)
    seg, out = {}, []
    for i in range(len(case.poses)):
        xyz = oracle.depth_to_cloud(depth[i], 8, sc.cx, sc.cy, sc.fx, sc.fy, 100.0)[0]
        lab = int(case.pose_label[i])
        tgt = case.obs_xyz[case.label_start[lab]:case.label_end[lab]]
        if len(xyz) == 0 or len(tgt) == 0:
            continue
        if lab not in seg:
            seg[lab] = oracle.covariances(tgt)
        out.append((xyz, oracle.covariances(xyz), tgt, seg[lab]))
    return out


def measure(pairs):
    q_total = q_diff = 0
    gap_max = 0.0
    it_diff, T_err, it_all, T_err_key = [], [], [], []
    for src, scov, tgt, tcov in pairs:
        T1, it1, tr = oracle.gicp_trace(src, scov, tgt, tcov)
        for k in range(len(tr)):  # the transform each linearisation searched from (tr[k]: state after iteration k)
            T = np.eye(4)
            if k > 0:
                T[:3, :3] = tr[k - 1, :9].reshape(3, 3)
                T[:3, 3] = tr[k - 1, 9:12]
            q = gref.query_f(T, src)
            jk = oracle.gicp_nn(q, tgt)
            je = gref.nearest_exact(q, tgt)
            q_total += len(q)
            d = je != jk
            q_diff += int(d.sum())
            if d.any():
                dd = q[d][:, None, :] - tgt[None, :, :]
                d2 = (dd[..., 0] * dd[..., 0] + dd[..., 1] * dd[..., 1]) + dd[..., 2] * dd[..., 2]
                r = np.arange(int(d.sum()))
                gap_max = max(gap_max, float((d2[r, jk[d]] - d2[r, je[d]]).max()))
        T2, it2 = gref.gicp(src, gref.covariances(src), tgt, gref.covariances(tgt))
        T3, it3 = gref.gicp(src, scov, tgt, tcov, nn=oracle.gicp_nn)  # the numpy chain on the key rule
        it_all.append(it1)
        it_diff.append(it1 != it2)
        T_err.append(float(np.abs(T1 - T2).max()))
        T_err_key.append(float(np.abs(T1 - T3).max()) if it1 == it3 else float("inf"))
    it_all = np.array(it_all)
    T_err = np.array(T_err)
    return {"poses": len(pairs), "at_150": int((it_all >= 150).sum()), "mean_iters": float(it_all.mean()),
            "queries": q_total, "queries_other_target": q_diff, "fraction_other_target": q_diff / max(q_total, 1),
            "max_sqdist_given_up_m2": gap_max,
            "poses_other_iteration_count": int(np.sum(it_diff)),
            "max_transform_diff_all": float(T_err.max()),
            "max_transform_diff_same_iters": float(T_err[~np.array(it_diff)].max()) if (~np.array(it_diff)).any() else None,
            "poses_transform_diff_over_1e-4": int((T_err > 1e-4).sum()),
            "key_rule_numpy_vs_oracle_max": float(np.max(T_err_key))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--poses-per-object", type=int, default=24)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    t0 = time.time()
    res = {"c3": measure(c3_pairs(a.poses_per_object, a.seed)), "poses_per_object": a.poses_per_object,
           "seed": a.seed}
    res["seconds"] = time.time() - t0
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
