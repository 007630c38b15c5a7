#!/usr/bin/env python
"""Latency of the heaviest GICP chains alone (round 6: why the 4-wave heavy-pose workgroups did not shorten the C3
launch's tail): the C3 candidates with the largest predicted cost (source points x targets), refined in a batch of
their own -- one pose per SIMD, nothing else on the GPU -- by the one-wave kernel (PCORE_GICP_KERNEL=n) and by
gicp_wide_kernel (8 waves splitting each pose's correspondence search, PCORE_GICP_KERNEL=w); per-chain time =
the GICP launch (pcore_get_stats gicp_ms).
    python tools/heavy_chain_probe.py [--top 16] [--out FILE.json]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from perception_amd import workloads  # noqa: E402

C3_NAMES = ["003_cracker_box", "005_tomato_soup_can", "006_mustard_bottle", "010_potted_meat_can", "024_bowl"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=16)
    ap.add_argument("--out")
    a = ap.parse_args()
    w = workloads.build(names=C3_NAMES, poses_per_model=10000)
    s = w.stride
    hs, ws = (w.scene.height + s - 1) // s, w.scene.width // s
    dbg = torch.empty((int(w.poses.shape[0]), hs, ws), dtype=torch.int32, device=w.poses.device)
    w.core.evaluate(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=s, dbg_zs=dbg)
    ns = (dbg > 0).sum(dim=(1, 2)).cpu().numpy()
    del dbg
    nt = w.pose_obs_total.cpu().numpy().astype(np.int64)
    top = np.argsort(-(ns * nt))[:a.top]
    idx = torch.from_numpy(top).to(w.poses.device)
    args = (w.poses[idx], w.pose_model[idx], w.pose_label[idx], w.pose_obs_total[idx])
    res = {"poses": [int(i) for i in top], "points": [int(ns[i]) for i in top], "targets": [int(nt[i]) for i in top]}
    for kern in ("n", "w", "n", "w"):
        os.environ["PCORE_GICP_KERNEL"] = kern
        adj, it, _, _, _ = w.core.evaluate_icp(*args, stride=s)
        st = w.core.stats()
        run = st["gicp_iterations_run"]
        res.setdefault(kern, []).append({"gicp_ms": st["gicp_ms"], "iterations_run": int(run),
                                         "iterations": [int(v) for v in it.cpu().numpy()]})
        print(kern, st["gicp_ms"], run, flush=True)
    s_ = json.dumps(res)
    print(s_)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s_ + "\n")


if __name__ == "__main__":
    main()
