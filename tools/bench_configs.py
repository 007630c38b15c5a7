#!/usr/bin/env python
"""Time the BASELINE.json configs other than the headline one on ONE GPU (per-GPU shares of the
multi-GPU configs).  Prints one JSON line per config.  Not the driver's bench (bench.py is).

  C1  1 mesh, 128 3-DoF table-top poses, render + GICP + re-render + score (cost type 0), 640x480 -- the GPU
      side of the workload bench.py's cpu_reference_path times on the reference's CPU/OMP path
  C2  1 mesh, 10k poses, render + score, 640x480
  C3  5 objects, 50k poses, render + GICP + re-render + score, 640x480 (+ argmin vs GT)
  C4  21 objects, 200k poses over 8 GPUs -> 25k poses per GPU, render + score
  C5  1 mesh, 1M poses at 1280x720 over 8 GPUs -> 125k poses per GPU, render + score
  C2scan_blob / C2scan_shell  C2 on a scan-like irregular mesh; C3scan  C3's flow on two scan meshes + the box
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from perception_amd import metrics  # noqa: E402
from perception_amd import synthetic as syn  # noqa: E402
from perception_amd import workloads  # noqa: E402
from perception_amd.model import to_eigen  # noqa: E402
from perception_amd._native import PCORE_KEY_NONE  # noqa: E402
from perception_amd.core import decode_keys  # noqa: E402

C3_NAMES = ["003_cracker_box", "005_tomato_soup_can", "006_mustard_bottle", "010_potted_meat_can", "024_bowl"]


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def run(name, names, per_model, cam, icp, steps, warmup):
    w = workloads.build(names=names, poses_per_model=per_model, cam=cam)
    n = int(w.poses.shape[0])
    dev = w.poses.device
    keys = torch.full((w.num_models,), PCORE_KEY_NONE, dtype=torch.int64, device=dev)
    if icp:
        out = (torch.empty((n, 16), dtype=torch.float32, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
               *(torch.empty(n, dtype=torch.float32, device=dev) for _ in range(3)))

        def step():
            keys.fill_(PCORE_KEY_NONE)
            adj, it, rc, oc, df = w.core.evaluate_icp(w.poses, w.pose_model, w.pose_label, w.pose_obs_total,
                                                      stride=w.stride, out=out)
            w.core.select(rc, oc, w.pose_model, w.num_models, keys=keys)
    else:
        out = tuple(torch.empty(n, dtype=torch.float32, device=dev) for _ in range(3))

        def step():
            keys.fill_(PCORE_KEY_NONE)
            workloads.step(w, out, keys)
    dt = timed(step, steps, warmup)
    cost, idx = decode_keys(keys)
    res = {"config": name, "poses": n, "models": w.num_models, "width": w.scene.width, "height": w.scene.height,
           "triangles": [int(c) for c in w.scene.bank.tris_model_count], "icp": icp, "s_per_step": dt, "poses_per_s": n / dt,
           "argmin_index": [int(i) for i in idx], "gt_index": [int(i) for i in w.gt_index],
           "argmin_cost": [int(c) for c in cost]}
    if icp:
        it = out[1].float()
        res["gicp_iters_mean"] = float(it.mean().item())
        res["gicp_iters_max"] = int(it.max().item())
        itn = out[1].cpu().numpy()
        edges = [1, 2, 5, 10, 20, 50, 100, 149, 150]
        res["gicp_iters_hist"] = {f"<={e}": int((itn <= e).sum()) for e in edges}
        res["gicp_iters_at_max"] = int((itn >= 150).sum())
        res["gicp_iters_p50_p90"] = [float(np.percentile(itn, 50)), float(np.percentile(itn, 90))]
    # pose accuracy of the selected poses against the synthetic ground truth (f3 metrics, on the GPU)
    final = (out[0] if icp else w.poses).cpu().numpy()
    errs_add, errs_adds = [], []
    for m in range(w.num_models):
        if idx[m] < 0:
            errs_add.append(np.inf)
            errs_adds.append(np.inf)
            continue
        est = to_eigen(final[idx[m]]).astype(np.float64)
        pts = np.unique(w.scene.bank.models[m].tris.reshape(-1, 3), axis=0)
        a, s_ = metrics.pose_distances(w.core, pts, w.scene.gt_poses[m][None], est[None])
        errs_add.append(float(a[0]))
        errs_adds.append(float(s_[0]))
    res["add_m"] = errs_add
    res["adds_m"] = errs_adds
    # the ground-truth candidates' own final costs (search_env.cpp:2022-2048 int conversion and filter), to explain a
    # winner other than the ground truth: a symmetric proxy (cylinder) renders the same at other yaws (ADD-S ~ 0)
    rcs, ocs = out[-3].cpu().numpy() if icp else out[0].cpu().numpy(), out[-2].cpu().numpy() if icp else out[1].cpu().numpy()
    gt_cost = []
    for g in w.gt_index:
        r, o = float(rcs[g]), float(ocs[g])
        gt_cost.append({"cost": int(np.float32(r) + np.float32(o)) if r >= 0 else -1, "rc": r, "oc": o,
                        "passes_filter": bool(r >= 0 and abs(int(r) - int(o)) < 30)})
    res["gt_candidate"] = gt_cost
    res["shapes"] = [syn.YCB_PROXIES[nm][0] if nm in syn.YCB_PROXIES else "?" for nm in names]
    res["adds_auc"] = metrics.compute_pose_metrics(np.array(errs_adds))["auc"]
    print(json.dumps(res), flush=True)
    del w
    torch.cuda.empty_cache()


def run_c1(steps, warmup, stride=4):
    """C1 on the GPU: the 128 3-DoF poses of workloads.c1_tabletop, scored against the whole observed cloud
    (3-DoF, no labels), with and without GICP."""
    from perception_amd.core import PoseCore
    from perception_amd.model import compute_proj
    dev = torch.device("cuda", 0)
    bank = syn.model_bank(["003_cracker_box"])
    core = PoseCore(0)
    core.upload_meshes(bank.tris, bank.tris_model_count)
    cam = syn.CAM_640
    core.set_camera(cam["width"], cam["height"], cam["fx"], cam["fy"], cam["cx"], cam["cy"],
                    compute_proj(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["width"], cam["height"]))
    W, H = cam["width"], cam["height"]
    core.set_observation(torch.zeros((H, W), dtype=torch.int32, device=dev), None,
                         torch.zeros((0, 3), dtype=torch.float32, device=dev), None, 0.01)
    c1 = workloads.c1_tabletop(workloads.gpu_render_fn(core, dev))
    sc = c1.scene
    xyz, _ = core.observed_cloud_bounded(torch.from_numpy(sc.depth_raw).to(dev), stride, sc.depth_factor)
    core.set_observation(torch.from_numpy(c1.src_depth_cm).to(dev), None, xyz, None, 0.0075)
    n = len(c1.poses)
    poses = torch.from_numpy(c1.poses).to(dev)
    pm = torch.zeros(n, dtype=torch.int32, device=dev)
    tot = torch.full((n,), float(xyz.shape[0]), dtype=torch.float32, device=dev)
    for icp in (False, True):
        if icp:
            fn = lambda: core.evaluate_icp(poses, pm, None, tot, cost_type=0, stride=stride,  # noqa: E731
                                           sensor_resolution=0.0075)
        else:
            fn = lambda: core.evaluate(poses, pm, None, tot, cost_type=0, stride=stride,  # noqa: E731
                                       sensor_resolution=0.0075)
        dt = timed(fn, steps, warmup)
        print(json.dumps({"config": "C1", "poses": n, "models": 1, "width": W, "height": H, "stride": stride,
                          "icp": icp, "s_per_step": dt, "poses_per_s": n / dt, "observed_points": int(xyz.shape[0])}),
              flush=True)
    # the launch-bound render + score as a captured HIP graph (PoseCore.capture_evaluate)
    replay, _ = core.capture_evaluate(poses, pm, None, tot, cost_type=0, stride=stride, sensor_resolution=0.0075)
    dt = timed(replay, steps, warmup)
    print(json.dumps({"config": "C1", "poses": n, "models": 1, "width": W, "height": H, "stride": stride,
                      "icp": False, "graph": True, "s_per_step": dt, "poses_per_s": n / dt,
                      "observed_points": int(xyz.shape[0])}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C1,C2,C3,C4,C5")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of the per-GPU pose count")
    a = ap.parse_args()
    sel = a.configs.split(",")
    sc = a.scale
    if "C1" in sel:
        run_c1(max(a.steps, 10), max(a.warmup, 2))
    if "C2" in sel:
        run("C2", ["003_cracker_box"], int(10000 * sc), syn.CAM_640, False, a.steps, a.warmup)
    if "C3" in sel:
        run("C3", C3_NAMES, int(10000 * sc), syn.CAM_640, True, a.steps, a.warmup)
    if "C4" in sel:
        run("C4/8", list(syn.YCB_PROXIES), int(25000 / 21 * sc), syn.CAM_640, False, a.steps, a.warmup)
    if "C5" in sel:
        run("C5/8", ["003_cracker_box"], int(125000 * sc), syn.CAM_1280, False, a.steps, a.warmup)
    # the scan-like irregular meshes (synthetic.scan_mesh) in C2's and C3's shape
    for nm in ("scan_blob", "scan_shell"):
        if "C2" + nm in sel:
            run("C2:" + nm, [nm], int(10000 * sc), syn.CAM_640, False, a.steps, a.warmup)
    if "C3scan" in sel:
        run("C3:scan", ["scan_blob", "scan_shell", "003_cracker_box"], int(10000 * sc), syn.CAM_640, True, a.steps,
            a.warmup)


if __name__ == "__main__":
    main()
