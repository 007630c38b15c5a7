#!/usr/bin/env python
"""Fused-kernel time against the batch size (C2 workload): does the last partial round of workgroups
(10,000 poses over 256 CUs x the occupancy) cost a visible tail?  Prints one JSON line per batch size
with the median HIP-event time of `evaluate` (stage COST) and the time per pose."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from perception_amd import workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1536,3072,4608,6144,7680,9216,10000,10752,12288,15360,20000")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    sizes = [int(x) for x in a.sizes.split(",")]
    w = workloads.build(poses_per_model=max(sizes))
    s = w.stride
    for n in sizes:
        args = (w.poses[:n], w.pose_model[:n], w.pose_label[:n], w.pose_obs_total)
        for _ in range(3):
            w.core.evaluate(*args, stride=s)
        torch.cuda.synchronize()
        ts = []
        stream = torch.cuda.current_stream()
        for _ in range(a.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            w.core.evaluate(*args, stride=s)
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        t = float(np.median(ts))
        print(json.dumps({"poses": n, "ms": t, "ns_per_pose": t * 1e6 / n}), flush=True)


if __name__ == "__main__":
    main()
