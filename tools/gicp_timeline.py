#!/usr/bin/env python
"""Timeline of one C3 GICP launch (a -DPCORE_GICP_TIMELINE build loaded with PCORE_LIB): per pose, when a wave dequeued
it and when it finished; per wave, its start and exit (100 MHz real-time clock).  Reports the launch span, the mean
number of busy waves against the resident maximum, when the queue ran dry (the last dequeue), the tail after it, and
the iteration counts of the poses that finish in that tail.
    PCORE_LIB=$PWD/build_ab/tl.so python tools/gicp_timeline.py [--out FILE.json]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from perception_amd import _native, workloads  # noqa: E402

C3_NAMES = ["003_cracker_box", "005_tomato_soup_can", "006_mustard_bottle", "010_potted_meat_can", "024_bowl"]
K_POSES, K_WAVES = 1 << 17, 1 << 14


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    a = ap.parse_args()
    w = workloads.build(names=C3_NAMES, poses_per_model=10000, device=0)
    lib = _native.load()
    fn = lib.pcore_debug_gicp_timeline
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    poses = np.zeros(2 * K_POSES, np.uint64)
    waves = np.zeros(2 * K_WAVES, np.uint64)
    nw = np.zeros(1, np.uint32)
    res = None
    for rep in range(2):  # the first call allocates and probes; the second is measured
        adj, it, rc, oc, df = w.core.evaluate_icp(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=w.stride)
        torch.cuda.synchronize()
        assert fn(poses.ctypes.data, waves.ctypes.data, nw.ctypes.data) == 0
    n = int(w.poses.shape[0])
    run = np.zeros(K_POSES, np.int32)
    lib.pcore_debug_gicp_timeline_run.argtypes = [ctypes.c_void_p]
    assert lib.pcore_debug_gicp_timeline_run(run.ctypes.data) == 0
    its_reported = it.cpu().numpy()
    its = run[:n].copy()  # the iterations each pose executed (a cycle exit reports 150 but runs fewer)
    ps = poses[:2 * n].reshape(n, 2).astype(np.int64)
    nwv = int(nw[0])
    ws = waves[:2 * nwv].reshape(nwv, 2).astype(np.int64)
    t0 = ws[:, 0].min()
    span = (ws[:, 1].max() - t0) / 100.0  # us
    # busy waves over time (1 us bins): a wave is busy from its start to its exit
    nb = int(span) + 1
    busy = np.zeros(nb + 1)
    for s, e in ws:
        busy[int((s - t0) / 100.0)] += 1
        busy[int((e - t0) / 100.0)] -= 1
    busy = np.cumsum(busy)[:nb]
    last_deq = (ps[:, 0].max() - t0) / 100.0
    tail_mask = (ps[:, 1] - t0) / 100.0 > last_deq
    pose_us = (ps[:, 1] - ps[:, 0]) / 100.0
    res = {"poses": n, "waves": nwv, "span_us": float(span), "mean_busy_waves": float(busy.mean()),
           "max_busy_waves": int(busy.max()), "busy_fraction": float(busy.mean() / busy.max()),
           "last_dequeue_us": float(last_deq), "tail_us": float(span - last_deq),
           "poses_finishing_in_tail": int(tail_mask.sum()),
           "tail_pose_iters_mean": float(its[tail_mask].mean()) if tail_mask.any() else None,
           "tail_pose_iters_at_150": int((its[tail_mask] >= 150).sum()),
           "pose_us_p50": float(np.percentile(pose_us, 50)), "pose_us_max": float(pose_us.max()),
           "us_per_iteration_mean": float((pose_us[its > 0] / its[its > 0]).mean()),
           "busy_below_90pct_us": float((busy < 0.9 * busy.max()).sum()),
           "busy_below_50pct_us": float((busy < 0.5 * busy.max()).sum()),
           "iterations_mean": float(its.mean()), "iterations_reported_mean": float(its_reported.mean()),
           "tail_pose_reported_at_150": int((its_reported[tail_mask] >= 150).sum()),
           "poses_run_150": int((its >= 150).sum())}
    # the longest poses: duration, iterations and source points (the stride-8 samples the cloud keeps)
    s8 = w.stride
    hs, ws8 = (w.scene.height + s8 - 1) // s8, w.scene.width // s8
    dbg = torch.empty((n, hs, ws8), dtype=torch.int32, device=w.poses.device)
    w.core.evaluate(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=s8, dbg_zs=dbg)
    ns = (dbg > 0).sum(dim=(1, 2)).cpu().numpy()
    nt = w.pose_obs_total.cpu().numpy().astype(np.int64)  # targets of the pose's label segment
    top = np.argsort(-pose_us)[:12]
    res["longest_poses"] = [{"pose": int(i), "us": float(pose_us[i]), "iterations": int(its[i]),
                             "iterations_reported": int(its_reported[i]), "points": int(ns[i]),
                             "targets": int(nt[i]), "start_us": float((ps[i, 0] - t0) / 100.0)} for i in top]
    end_us = (ps[:, 1] - t0) / 100.0
    res["last_poses"] = [{"pose": int(i), "start_us": float((ps[i, 0] - t0) / 100.0), "end_us": float(end_us[i]),
                          "iterations": int(its[i]), "points": int(ns[i]), "targets": int(nt[i])}
                         for i in np.argsort(-end_us)[:8]]
    res["poses_over_512_points"] = int((ns > 512).sum())
    res["points_mean"] = float(ns.mean())
    res["segment_targets"] = sorted(set(int(v) for v in nt))
    # time per pose against its predicted cost (points x targets) and iterations
    res["us_per_iteration_by_targets"] = {str(v): float((pose_us[(nt == v) & (its > 0)] / its[(nt == v) & (its > 0)]).mean())
                                          for v in sorted(set(int(v) for v in nt))}
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
