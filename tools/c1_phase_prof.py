#!/usr/bin/env python
"""Per-phase shader clocks of gicp_wide_kernel on C1 (build with -DPCORE_GICP_PROFILE, load with PCORE_LIB): wave 0's
clocks per pose-iteration in the all-wave correspondence search (to the barrier), the contributions, the 28-term tree
and the LM iteration (solves, se3_exp + compose, trial errors, decisions)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from perception_amd import _native, synthetic as syn, workloads  # noqa: E402
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
    xyz, _ = core.observed_cloud_bounded(torch.from_numpy(c1.scene.depth_raw).to(dev), stride, c1.scene.depth_factor)
    core.set_observation(torch.from_numpy(c1.src_depth_cm).to(dev), None, xyz, None, 0.0075)
    n = len(c1.poses)
    poses = torch.from_numpy(c1.poses).to(dev)
    pm = torch.zeros(n, dtype=torch.int32, device=dev)
    tot = torch.full((n,), float(xyz.shape[0]), dtype=torch.float32, device=dev)
    fn = _native.load().pcore_debug_gicp_profile
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 8)()
    core.evaluate_icp(poses, pm, None, tot, cost_type=0, stride=stride, sensor_resolution=0.0075)
    torch.cuda.synchronize()
    fn(buf, 1)
    _, iters, _, _, _ = core.evaluate_icp(poses, pm, None, tot, cost_type=0, stride=stride, sensor_resolution=0.0075)
    torch.cuda.synchronize()
    fn(buf, 0)
    it = iters.cpu().numpy()
    total = int(it.sum())
    names = ["search (all waves)", "contributions", "reduction", "LM iteration", "  solves", "  se3 + compose",
             "  trial errors", "  decisions"]
    print("pose-iterations", total, "mean iters", it.mean(), "max", it.max())
    for k in range(8):
        print(f"{names[k]:20s} {buf[k] / max(total, 1):10.0f} clk per pose-iteration")


if __name__ == "__main__":
    main()
