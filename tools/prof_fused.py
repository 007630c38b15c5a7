#!/usr/bin/env python
"""Run the C2 workload's fused kernel a few times (for rocprofv3 counter / trace collection)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from perception_amd import workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--poses", type=int, default=10000)
    ap.add_argument("--icp", action="store_true")
    ap.add_argument("--c3", action="store_true", help="the 5-object C3 scene")
    ap.add_argument("--iters-json", default=None, help="write the GICP iterations of the last call here (--icp)")
    ap.add_argument("--mesh", default="003_cracker_box", help="the single mesh of the C2 workload (e.g. scan_blob)")
    a = ap.parse_args()
    names = ["003_cracker_box", "005_tomato_soup_can", "006_mustard_bottle", "010_potted_meat_can",
             "024_bowl"] if a.c3 else [a.mesh]
    w = workloads.build(names=names, poses_per_model=a.poses)
    n = int(w.poses.shape[0])
    its = None
    for _ in range(a.iters):
        if a.icp:
            _, its, _, _, _ = w.core.evaluate_icp(w.poses, w.pose_model, w.pose_label, w.pose_obs_total,
                                                  stride=w.stride)
        else:
            w.core.evaluate(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=w.stride)
        torch.cuda.synchronize()  # steady state: the next call sees this call's window histogram
    if a.iters_json and its is not None:
        import json
        st = w.core.stats()  # pose_iterations: the executed ones (the cycle exits' remaining iterations are not run)
        with open(a.iters_json, "w") as f:
            json.dump({"poses": n, "pose_iterations": int(st["gicp_iterations_run"]),
                       "pose_iterations_reported": int(its.sum().item()), "cycle_exits": int(st["gicp_cycle_exits"]),
                       "gicp_launches_per_call": 1}, f)
    print("done", n)


if __name__ == "__main__":
    main()
