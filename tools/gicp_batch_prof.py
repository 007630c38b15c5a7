#!/usr/bin/env python
"""Wave clocks of gicp_batch_kernel (build with -DPCORE_GICP_PROFILE, load with PCORE_LIB) on C3: point passes vs LM
lane steps, rounds and passes per pose-iteration, plus the GICP call's own time."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from perception_amd import _native, workloads  # noqa: E402


def main():
    names = ["003_cracker_box", "005_tomato_soup_can", "006_mustard_bottle", "010_potted_meat_can", "024_bowl"]
    w = workloads.build(names=names, poses_per_model=10000)
    lib = _native.load()
    fn = lib.pcore_debug_gicp_profile
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 9)()
    w.core.evaluate_icp(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=w.stride)
    torch.cuda.synchronize()
    fn(buf, 1)
    adj, iters, rc, oc, df = w.core.evaluate_icp(w.poses, w.pose_model, w.pose_label, w.pose_obs_total,
                                                 stride=w.stride)
    torch.cuda.synchronize()
    st = w.core.stats()
    fn(buf, 0)
    total = int(iters.cpu().numpy().sum())
    print(f"pose-iterations {total}  gicp {st['gicp_ms']:.3f} ms")
    print(f"passes {buf[3]} ({buf[3] / total:.3f} per pose-iteration), rounds {buf[2]}, live slots per round "
          f"{buf[3] / max(buf[2], 1):.2f}")
    print(f"pass clocks per pass {buf[0] / max(buf[3], 1):.0f}, LM step clocks per round {buf[1] / max(buf[2], 1):.0f}")
    print(f"per pose-iteration: passes {buf[0] / total:.0f} + LM {buf[1] / total:.0f} wave clocks")
    for k, n in ((4, "pass setup (pose, history)"), (5, "trial error"), (6, "search / history read"),
                 (7, "contributions"), (8, "reductions")):
        print(f"  {n:28s} {buf[k] / total:8.0f} per pose-iteration")


if __name__ == "__main__":
    main()
