#!/usr/bin/env python
"""The poses that end C3's GICP launch (profiles/r06s/tl_help*.json: 23-36-point clouds on the 32-target segment,
150 executed iterations): why does the cycle exit not stop them?  On the bench workload (a GPU builds it), the small
clouds of the smallest segment are traced by the oracle's GICP on the CPU (full length, no exit); the exit rule is
simulated on each trace with 32 / 64 / 128 lags (tools/cycle_exit_sim.simulate), and the capped poses that no lag
count stops are characterised: the first recurrence lag of their last float transform and their LM flags.
    python tools/tail_pose_trace.py [--max-points 40] [--poses 200] [--out FILE.json]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

C3_NAMES = ["003_cracker_box", "005_tomato_soup_can", "006_mustard_bottle", "010_potted_meat_can", "024_bowl"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-points", type=int, default=40)
    ap.add_argument("--poses", type=int, default=200)
    ap.add_argument("--out")
    a = ap.parse_args()
    import cycle_exit_sim as S
    import oracle
    from perception_amd import workloads

    w = workloads.build(names=C3_NAMES, poses_per_model=10000)
    sc = w.scene
    s8 = w.stride
    dbg = torch.empty((w.poses.shape[0], (sc.height + s8 - 1) // s8, sc.width // s8), dtype=torch.int32,
                      device=w.poses.device)
    w.core.evaluate(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=s8, dbg_zs=dbg)
    ns = (dbg > 0).sum(dim=(1, 2)).cpu().numpy()
    nt = w.pose_obs_total.cpu().numpy().astype(np.int64)
    small_seg = int(nt.min())
    cand = np.nonzero((nt == small_seg) & (ns > 10) & (ns <= a.max_points))[0]
    cand = np.random.default_rng(3).choice(cand, min(a.poses, len(cand)), replace=False)
    xyz = w.obs_xyz.cpu().numpy()
    lab = w.obs_label.cpu().numpy()
    order = np.argsort(lab, kind="stable")
    oxyz, olab = xyz[order], lab[order]
    poses = w.poses.cpu().numpy()
    pm = w.pose_model.cpu().numpy()
    res = {"segment_targets": small_seg, "traced": 0, "capped": 0, "exits": {}, "unstopped": []}
    covs = {}
    traces = []
    for i in cand:
        L = int(pm[i])
        depth = oracle.render_depth(sc.bank.tris, sc.bank.tris_model_count, poses[i:i + 1], pm[i:i + 1], pm[i:i + 1],
                                    sc.width, sc.height, sc.proj, sc.src_depth_cm, sc.mask, 1.0)
        src = oracle.depth_to_cloud(depth[0], s8, sc.cx, sc.cy, sc.fx, sc.fy, 100.0)[0]
        tgt = oxyz[olab == L]
        if len(src) == 0 or len(tgt) == 0:
            continue
        if L not in covs:
            covs[L] = oracle.covariances(tgt)
        T, it, tr = oracle.gicp_trace(src, oracle.covariances(src), tgt, covs[L])
        traces.append((int(i), len(src), T, it, tr))
    res["traced"] = len(traces)
    cap = [t for t in traces if t[3] >= 150]
    res["capped"] = len(cap)
    stop = {}
    for lags in (32, 64, 128):
        stop[lags] = set()
        for i, n, T, it, tr in cap:
            k, _ = S.simulate(tr, it, 8, True, True, lags)
            if k:
                stop[lags].add(i)
        res["exits"][str(lags)] = len(stop[lags])
    for i, n, T, it, tr in cap:
        if i in stop[128]:
            continue
        X = tr[:, :12].astype(np.float32).view(np.uint32)
        rep = [k for k in range(1, min(140, len(X) - 1)) if np.array_equal(X[-1 - k], X[-1])]
        res["unstopped"].append({"pose": i, "points": n, "first_repeat_lags": rep[:3],
                                 "trials_last10": tr[-10:, 13].astype(int).tolist(),
                                 "flags_last10": tr[-10:, 14].astype(int).tolist()})
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
