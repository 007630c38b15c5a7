#!/usr/bin/env python
"""Time the fused window launch under every LDS tile tier (PCORE_FUSED_TIER) and the automatic choice, on the
render + score configs (C2, C4 share, C5 share), and print the window histogram the launch published
(pcore_get_tile_info).  One JSON line per (config, tier).  Measurement tool for the tier chooser (DESIGN.md
"Pose windows"); not the driver's bench."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from perception_amd import synthetic as syn  # noqa: E402
from perception_amd import workloads  # noqa: E402
from perception_amd._native import PCORE_KEY_NONE  # noqa: E402

CONFIGS = {
    "C2": (["003_cracker_box"], 10000, syn.CAM_640),
    "C4/8": (list(syn.YCB_PROXIES), 25000 // 21, syn.CAM_640),
    "C5/8": (["003_cracker_box"], 125000, syn.CAM_1280),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2,C4/8,C5/8")
    ap.add_argument("--tiers", default="auto,0,1,2,3,4")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    for name in a.configs.split(","):
        names, per_model, cam = CONFIGS[name]
        w = workloads.build(names=names, poses_per_model=per_model, cam=cam)
        n = int(w.poses.shape[0])
        dev = w.poses.device
        keys = torch.full((w.num_models,), PCORE_KEY_NONE, dtype=torch.int64, device=dev)
        out = tuple(torch.empty(n, dtype=torch.float32, device=dev) for _ in range(3))
        for tier in a.tiers.split(","):
            if tier == "auto":
                os.environ.pop("PCORE_FUSED_TIER", None)
            else:
                os.environ["PCORE_FUSED_TIER"] = tier
            for _ in range(3):  # the automatic choice needs a published histogram of an earlier launch
                workloads.step(w, out, keys)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                workloads.step(w, out, keys)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.steps
            print(json.dumps({"config": name, "tier": tier, "poses": n, "ms_per_step": dt * 1e3,
                              "poses_per_s": n / dt, "tile": w.core.tile_info()}), flush=True)
        os.environ.pop("PCORE_FUSED_TIER", None)
        del w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
