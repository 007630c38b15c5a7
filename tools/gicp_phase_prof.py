#!/usr/bin/env python
"""Per-phase shader clocks of gicp_kernel (build with -DPCORE_GICP_PROFILE, load with PCORE_LIB):
linearisation (correspondence search + contributions) / 28-term wave reduction / LM iteration (damped solves,
se3_exp, the trials' error sums), per pose-iteration."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from perception_amd import _native, workloads  # noqa: E402


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--c3", action="store_true", help="the 5-object C3 scene instead of C2's single object")
    ap.add_argument("--poses", type=int, default=10000, help="poses per model")
    ap.add_argument("--max-ns", type=int, default=0,
                    help="only the poses of at most this many source points, run alone (an idle GPU: the chains' latency)")
    a = ap.parse_args()
    names = ["003_cracker_box", "005_tomato_soup_can", "006_mustard_bottle", "010_potted_meat_can",
             "024_bowl"] if a.c3 else ["003_cracker_box"]
    w = workloads.build(names=names, poses_per_model=a.poses)
    if a.max_ns:
        s8 = w.stride
        dbg = torch.empty((w.poses.shape[0], (w.scene.height + s8 - 1) // s8, w.scene.width // s8), dtype=torch.int32,
                          device=w.poses.device)
        w.core.evaluate(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=s8, dbg_zs=dbg)
        ns = (dbg > 0).sum(dim=(1, 2))
        sel = torch.nonzero((ns > 0) & (ns <= a.max_ns)).flatten()[:512]
        w.poses, w.pose_model = w.poses[sel].contiguous(), w.pose_model[sel].contiguous()
        w.pose_label, w.pose_obs_total = w.pose_label[sel].contiguous(), w.pose_obs_total[sel].contiguous()
        print("poses of <=", a.max_ns, "points:", int(sel.numel()), "mean points", float(ns[sel].float().mean()))
    lib = _native.load()
    fn = lib.pcore_debug_gicp_profile
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 10)()
    w.core.evaluate_icp(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=w.stride)
    torch.cuda.synchronize()
    fn(buf, 1)
    adj, iters, rc, oc, df = w.core.evaluate_icp(w.poses, w.pose_model, w.pose_label, w.pose_obs_total,
                                                 stride=w.stride)
    torch.cuda.synchronize()
    fn(buf, 0)
    it = iters.cpu().numpy()
    st = w.core.stats()
    if a.max_ns:  # every pose on its own wave: the launch lasts about the longest chain
        print(f"gicp_ms {st['gicp_ms']:.3f}; per iteration of the longest chain {1e3 * st['gicp_ms'] / max(it.max(), 1):.2f} us")
    # one linearisation + one LM iteration per executed iteration (a cycle exit reports 150 but runs fewer)
    total = int(buf[9])  # the executed pose-iterations of the profiled poses (a PCORE_GICP_PROF_MIN_NS build: the large ones)
    names = ["search", "contributions", "reduction", "LM iteration", "  solves", "  se3 + compose", "  trial errors",
             "  decisions"]
    print("pose-iterations", total, "mean iters", it.mean(), "max", it.max())
    for k in range(8):
        print(f"{names[k]:14s} {buf[k] / max(total, 1):10.0f} clk per pose-iteration")
    print(f"correspondence history reuse: {buf[8]} of {total} pose-iterations ({buf[8] / max(total, 1):.3f})")


if __name__ == "__main__":
    main()
