#!/usr/bin/env python
"""Per-phase shader clocks of fused_cost_kernel (build with -DPCORE_FUSED_PROFILE, load with PCORE_LIB):
wave-clocks per pose in setup / vertex stage / triangle windows / fragment batches / end-of-raster barrier /
phase 2 / phase 3, summed over the 4 waves of a pose's workgroup (so they include the time a wave waits
while the SIMD runs other waves)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from perception_amd import _native, workloads  # noqa: E402

NAMES = ["setup", "vertex", "tri_windows", "fragments", "raster_barrier", "phase2", "phase3"]


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--poses", type=int, default=10000)
    ap.add_argument("--cam", default="640")
    a = ap.parse_args()
    from perception_amd import synthetic as syn
    w = workloads.build(poses_per_model=a.poses, cam=syn.CAM_640 if a.cam == "640" else syn.CAM_1280)
    lib = _native.load()
    fn = lib.pcore_debug_fused_profile
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 8)()
    for _ in range(2):
        w.core.evaluate(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=w.stride)
    torch.cuda.synchronize()
    fn(buf, 1)
    reps = 3
    for _ in range(reps):
        w.core.evaluate(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=w.stride)
    torch.cuda.synchronize()
    fn(buf, 0)
    n = int(w.poses.shape[0]) * reps
    tot = sum(buf[k] for k in range(7))
    res = {NAMES[k]: {"wave_clk_per_pose": buf[k] / n, "frac": buf[k] / max(tot, 1)} for k in range(7)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
