#!/usr/bin/env python
"""How many of the fused kernel's raster steps could be skipped whole, estimated on the CPU
before building anything.  A step is one batch of <= 64 triangles of a wave's vertex-ring stream
(perception_amd/csrc/pcore_streams.h, tools/stream_stats.cpp stream_steps); C2's box proxy has 195 of them per pose.
For every step and candidate pose this counts whether
  aabb:   the conservative sample window of the step -- the model-space bounding box of its triangles' vertices, its
          8 corners through the pose and compute_proj, +-2 px -- holds no stride-s sample (what a per-step test in the
          kernel could check before the triangle stage), or
  exact:  none of its triangles' own sample windows (the kernel's per-triangle window, +-1 px) holds a sample
          (the upper bound of any per-step skip).
A step whose window reaches behind the camera is never counted.  The poses are C2-style candidates around the GT
(tests/helpers.SceneCase).
    python tools/step_skip_estimate.py [--poses 300] [--stride 8]"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def stream_steps(tris):
    lib_path = os.path.join(ROOT, "tools", "bin", "libstreamstats.so")
    if not os.path.exists(lib_path):
        os.makedirs(os.path.dirname(lib_path), exist_ok=True)
        subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", os.path.join(ROOT, "tools", "stream_stats.cpp"),
                        "-o", lib_path], check=True)
    lib = ctypes.CDLL(lib_path)
    T = len(tris)
    cap = 4 * T // 64 + 64
    out = np.zeros(64 * cap, np.int32)
    t = np.ascontiguousarray(tris, np.float32).reshape(-1)
    n = lib.stream_steps(t.ctypes.data_as(ctypes.c_void_p), T, 4, 4, 2, 1, out.ctypes.data_as(ctypes.c_void_p), cap)
    return out[:64 * n].reshape(n, 64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--poses", type=int, default=300)
    ap.add_argument("--stride", type=int, default=8)
    a = ap.parse_args()
    from tests.helpers import SceneCase

    case = SceneCase(("003_cracker_box",), n_poses=a.poses)
    sc = case.scene
    W, H, s = sc.width, sc.height, a.stride
    tris = sc.bank.tris.reshape(-1, 3, 3).astype(np.float64)
    steps = stream_steps(sc.bank.tris)
    P = np.asarray(sc.proj, np.float64).reshape(4, 4)
    nx, ny = W // s, (H + s - 1) // s

    def has_sample(x0, x1, y0, y1):
        """a stride-s sample (column kx*s, image row ky*s; image row = H-1-screen y) inside the screen box"""
        kx0, kx1 = np.maximum(0, np.ceil(x0 / s)), np.minimum(nx - 1, np.floor(x1 / s))
        r0, r1 = H - 1 - y1, H - 1 - y0
        ky0, ky1 = np.maximum(0, np.ceil(r0 / s)), np.minimum(ny - 1, np.floor(r1 / s))
        return (kx1 >= kx0) & (ky1 >= ky0)

    def screen(cam):
        z = cam[..., 2]
        px = cam @ P[0, :3] + P[0, 3]
        py = cam @ P[1, :3] + P[1, 3]
        return px / z * W / 2 + W / 2, py / z * H / 2 + H / 2, z

    skip_aabb = skip_exact = total = 0
    for i in range(len(case.poses)):
        m = case.poses[i].astype(np.float64).reshape(4, 4)
        for row in steps:
            tid = row[row >= 0]
            if not len(tid):
                continue
            total += 1
            v = tris[tid].reshape(-1, 3)
            lo, hi = v.min(0), v.max(0)
            c = np.array([[x, y, z] for x in (lo[0], hi[0]) for y in (lo[1], hi[1]) for z in (lo[2], hi[2])])
            sx, sy, z = screen(c @ m[:3, :3].T + m[:3, 3])
            if z.min() > 1 and not has_sample(sx.min() - 2, sx.max() + 2, sy.min() - 2, sy.max() + 2):
                skip_aabb += 1
            tx, ty, tz = screen(tris[tid] @ m[:3, :3].T + m[:3, 3])  # (n, 3) per vertex
            if tz.min() > 1 and not has_sample(tx.min(1) - 1, tx.max(1) + 1, ty.min(1) - 1, ty.max(1) + 1).any():
                skip_exact += 1
    res = {"poses": len(case.poses), "steps_per_pose": int(len(steps)), "step_visits": total,
           "skippable_aabb_frac": skip_aabb / total, "skippable_exact_frac": skip_exact / total, "stride": s,
           "build_threshold": 0.25}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
