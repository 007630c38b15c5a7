#!/usr/bin/env python
"""Fused COST kernel time against the batch size (C2 scene): slope (steady-state ns per pose) and intercept
(the launch's fill + drain), from HIP events around stage COST on the stream it runs on."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from perception_amd import workloads  # noqa: E402


def main():
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1536,3072,5000,10000,20000,40000").split(",")]
    w = workloads.build(poses_per_model=max(sizes))
    res = []
    stream = torch.cuda.current_stream()
    for n in sizes:
        args = (w.poses[:n], w.pose_model[:n], w.pose_label[:n], w.pose_obs_total[:n])
        for _ in range(3):
            w.core.evaluate(*args, stride=w.stride)
        torch.cuda.synchronize()
        ts = []
        for _ in range(10):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            w.core.evaluate(*args, stride=w.stride)
            b.record(stream)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        res.append((n, float(np.median(ts))))
    x = np.array([r[0] for r in res], float)
    y = np.array([r[1] for r in res], float)
    big = x >= 5000
    slope, icpt = np.polyfit(x[big], y[big], 1)
    print(json.dumps({"points_ms": res, "ns_per_pose": slope * 1e6, "intercept_us": icpt * 1e3}))


if __name__ == "__main__":
    main()
