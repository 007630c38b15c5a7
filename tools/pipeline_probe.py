#!/usr/bin/env python
"""Probe: C2 steps on one stream / one context against consecutive steps alternating over two contexts on two
HIP streams (a step's drain overlaps the next step's fill)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from perception_amd import workloads  # noqa: E402
from perception_amd.core import PoseCore  # noqa: E402


def main():
    w = workloads.build()
    sc, dev = w.scene, w.poses.device
    c2 = PoseCore(dev.index)
    c2.upload_meshes(sc.bank.tris, sc.bank.tris_model_count, sc.bank.colors)
    c2.set_camera(sc.width, sc.height, sc.fx, sc.fy, sc.cx, sc.cy, sc.proj)
    c2.set_observation(torch.from_numpy(sc.src_depth_cm).to(dev), torch.from_numpy(sc.mask).to(dev), w.obs_xyz,
                       w.obs_label, 0.01)
    cores = [w.core, c2]
    streams = [torch.cuda.current_stream(), torch.cuda.Stream(dev)]
    n = int(w.poses.shape[0])
    outs = [tuple(torch.empty(n, dtype=torch.float32, device=dev) for _ in range(3)) for _ in range(2)]
    args = (w.poses, w.pose_model, w.pose_label, w.pose_obs_total)
    res = {}
    for mode in ("one", "two", "one", "two"):
        k = 1 if mode == "one" else 2
        for i in range(6):
            cores[i % k].evaluate(*args, stride=w.stride, out=outs[i % k], stream=streams[i % k])
        torch.cuda.synchronize()
        steps = 40
        t0 = time.perf_counter()
        for i in range(steps):
            j = i % k
            if j != 0:
                streams[j].wait_stream(streams[0]) if False else None
            cores[j].evaluate(*args, stride=w.stride, out=outs[j], stream=streams[j])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res.setdefault(mode, []).append(dt / steps * 1e3)
    ok = all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))
    print(json.dumps({"ms_per_step": res, "outputs_equal": ok}))


if __name__ == "__main__":
    main()
