#!/usr/bin/env python
"""C1's GICP in numbers: the 128 3-DoF poses' rendered-cloud sizes (stride 4), GICP iterations, and the GICP stage
time of gicp_wide_kernel (8 waves per pose) against gicp_kernel (one wave per pose), from pcore_get_stats."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from perception_amd import synthetic as syn, workloads  # noqa: E402
from perception_amd.core import PoseCore  # noqa: E402
from perception_amd.model import compute_proj  # noqa: E402


def main(stride=4):
    dev = torch.device("cuda", 0)
    bank = syn.model_bank(["003_cracker_box"])
    core = PoseCore(0)
    core.upload_meshes(bank.tris, bank.tris_model_count)
    cam = syn.CAM_640
    W, H = cam["width"], cam["height"]
    core.set_camera(W, H, cam["fx"], cam["fy"], cam["cx"], cam["cy"],
                    compute_proj(cam["fx"], cam["fy"], cam["cx"], cam["cy"], W, H))
    core.set_observation(torch.zeros((H, W), dtype=torch.int32, device=dev), None,
                         torch.zeros((0, 3), dtype=torch.float32, device=dev), None, 0.01)
    c1 = workloads.c1_tabletop(workloads.gpu_render_fn(core, dev))
    sc = c1.scene
    xyz, _ = core.observed_cloud_bounded(torch.from_numpy(sc.depth_raw).to(dev), stride, sc.depth_factor)
    src = torch.from_numpy(c1.src_depth_cm).to(dev)
    core.set_observation(src, None, xyz, None, 0.0075)
    n = len(c1.poses)
    poses = torch.from_numpy(c1.poses).to(dev)
    pm = torch.zeros(n, dtype=torch.int32, device=dev)
    tot = torch.full((n,), float(xyz.shape[0]), dtype=torch.float32, device=dev)
    depth = core.render(poses, pm, None)
    _, pose_of, _ = core.depth_to_cloud(depth, stride, 100.0)
    counts = np.bincount(pose_of.cpu().numpy(), minlength=n)
    out = {"poses": n, "observed_points": int(xyz.shape[0]),
           "src_points": {"mean": float(counts.mean()), "max": int(counts.max()), "min": int(counts.min())}}
    for kern in ("w", "n"):
        os.environ["PCORE_GICP_KERNEL"] = kern
        res = None
        times = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = core.evaluate_icp(poses, pm, None, tot, cost_type=0, stride=stride, sensor_resolution=0.0075)
            st = core.stats()
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t0, st["gicp_ms"]))
        it = res[1].cpu().numpy()
        out["wide" if kern == "w" else "narrow"] = {
            "call_ms": round(1e3 * min(t for t, _ in times), 2), "gicp_ms": round(min(g for _, g in times), 2),
            "iters_mean": float(it.mean()), "iters_max": int(it.max()), "at_150": int((it >= 150).sum())}
    del os.environ["PCORE_GICP_KERNEL"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
