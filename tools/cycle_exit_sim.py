#!/usr/bin/env python
"""Simulate the GICP cycle exit on oracle traces of C3-style candidates, before building it.

For every candidate the oracle runs the full spec (no exit) with its per-iteration trace.  The simulation then applies
the exit rule to the trace: at the top of iteration k, if the float linearisation transforms T_f(j) = float(x_{j-1})
of the last W iterations all recur at the same smallest lag p (T_f(j) == T_f(j - p), bit for bit, p <= 16) and the LM
steps that produced them were all accepted at their first trial with rho >= 1/2 and an inert damping (lambda changes
no diagonal entry of H), the pose stops and reports T_f of the cycle member at iteration max_iter + 1.  It prints, per
W, how many exits would happen, how many iterations they save, and how many predicted results differ from the full
run (float transform bits, reported iteration counts).
    python tools/cycle_exit_sim.py [--per-object 200] [--seed 7] [--out FILE.json]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from tests.helpers import SceneCase  # noqa: E402

C3_NAMES = ("003_cracker_box", "004_sugar_box", "005_tomato_soup_can", "006_mustard_bottle", "010_potted_meat_can")
MAX_ITER = 150
LAGS = 32  # pcore_gicp_math.h kCycleLags


def candidates(per_object, seed):
    case = SceneCase(names=C3_NAMES, n_poses=per_object, seed=seed)
    sc = case.scene
    depth = oracle.render_depth(sc.bank.tris, sc.bank.tris_model_count, case.poses, case.pose_model, case.pose_label,
                                sc.width, sc.height, sc.proj, sc.src_depth_cm, sc.mask, 1.0)
    seg = {}
    for i in range(len(case.poses)):
        xyz = oracle.depth_to_cloud(depth[i], 8, sc.cx, sc.cy, sc.fx, sc.fy, 100.0)[0]
        lab = int(case.pose_label[i])
        tgt = case.obs_xyz[case.label_start[lab]:case.label_end[lab]]
        if len(xyz) == 0 or len(tgt) == 0:
            continue
        if lab not in seg:
            seg[lab] = oracle.covariances(tgt)
        yield xyz, oracle.covariances(xyz), tgt, seg[lab]


def simulate(tr, it, W, need_inert=True, need_rho=True, lags=LAGS):
    """(exit iteration or 0, predicted final float transform bits (12,) or None)"""
    X = tr[:, :12].astype(np.float32).view(np.uint32)  # float(x_k), k = 1..it (row k - 1)
    ident = np.array([1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0], np.float32).view(np.uint32)
    Tf = np.vstack([ident, X])  # Tf[j - 1] = T_f(j) = float(x_{j - 1}), j = 1..it + 1
    ok = (tr[:, 13] == 1) & (tr[:, 15] == 0)
    if need_inert:
        ok &= (tr[:, 14].astype(int) & 1) == 1
    if need_rho:
        ok &= (tr[:, 14].astype(int) & 2) == 2
    lag = np.zeros(it + 2, np.int64)
    run = 0
    okrun = 0
    for k in range(1, it + 1):  # top of iteration k: T_f(k) known, steps 1..k-1 done
        okrun = okrun + 1 if (k >= 2 and ok[k - 2]) else 0
        p = 0
        for q in range(1, min(lags, k - 1) + 1):
            if np.array_equal(Tf[k - 1], Tf[k - 1 - q]):
                p = q
                break
        lag[k] = p
        run = run + 1 if (p > 0 and p == lag[k - 1]) else (1 if p > 0 else 0)
        if p > 0 and run >= W and okrun >= W:
            jstar = MAX_ITER + 1
            jp = k - ((k - jstar) % p)
            return k, Tf[jp - 1]
    return 0, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-object", type=int, default=200)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--out")
    a = ap.parse_args()
    traces = []
    for src, scov, tgt, tcov in candidates(a.per_object, a.seed):
        T, it, tr = oracle.gicp_trace(src, scov, tgt, tcov)
        traces.append((T, it, tr))
    iters = np.array([t[1] for t in traces])
    res = {"candidates": len(traces), "at_150": int((iters >= MAX_ITER).sum()), "iterations": int(iters.sum()),
           "variants": []}
    for W, inert, rhoc, lags in [(2, True, True, 16), (3, True, True, 16), (4, True, True, 16), (6, True, True, 16),
                                 (8, True, True, 16), (12, True, True, 16), (4, False, True, 16), (4, False, False, 16),
                                 (8, False, False, 16), (8, True, True, 32), (8, True, True, 64), (16, True, True, 32),
                                 (16, True, True, 64)]:
        n_exit = saved = wrong_T = wrong_it = 0
        for T, it, tr in traces:
            k, pred = simulate(tr, it, W, inert, rhoc, lags)
            if not k:
                continue
            n_exit += 1
            saved += it - (k - 1)
            final = np.concatenate([T[:3, :3].reshape(-1), T[:3, 3]]).astype(np.float32).view(np.uint32)
            if it != MAX_ITER:
                wrong_it += 1
            if not np.array_equal(final, pred):
                wrong_T += 1
        v = {"W": W, "lags": lags, "need_inert": inert, "need_rho_half": rhoc, "exits": n_exit, "iterations_saved": int(saved),
             "saved_frac": saved / max(1, int(iters.sum())), "wrong_transform": wrong_T, "wrong_iterations": wrong_it}
        res["variants"].append(v)
        print(v, flush=True)
    s = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
