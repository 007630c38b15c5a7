#!/usr/bin/env python
"""Where C3's GICP time goes: per pose, the scan work of its iterations (iterations x 64-point rounds x
target quads), the heaviest poses against the average work per wave (3 waves per SIMD on the device)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from perception_amd import workloads  # noqa: E402


def main():
    names = ["003_cracker_box", "005_tomato_soup_can", "006_mustard_bottle", "010_potted_meat_can", "024_bowl"]
    w = workloads.build(names=names, poses_per_model=10000)
    n = int(w.poses.shape[0])
    s = w.stride
    hs, ws = (w.scene.height + s - 1) // s, w.scene.width // s
    ns = np.zeros(n, np.int64)
    for lo in range(0, n, 5000):
        hi = min(n, lo + 5000)
        dbg = torch.empty((hi - lo, hs, ws), dtype=torch.int32, device=w.poses.device)
        w.core.evaluate(w.poses[lo:hi], w.pose_model[lo:hi], w.pose_label[lo:hi], w.pose_obs_total[lo:hi],
                        stride=s, dbg_zs=dbg)
        ns[lo:hi] = (dbg > 0).sum(dim=(1, 2)).cpu().numpy()
    _, iters, _, _, _ = w.core.evaluate_icp(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=s)
    it = iters.cpu().numpy().astype(np.int64)
    nt = np.bincount(w.obs_label.cpu().numpy(), minlength=w.num_models)[w.pose_label.cpu().numpy()]
    work = (it + 1) * ((ns + 63) // 64) * ((nt + 3) // 4)
    waves = 3 * 4 * 256
    order = np.argsort(-work)
    print("poses", n, "mean iters %.1f" % it.mean(), "at 150: %d" % (it == 150).sum(),
          "ns mean %.0f max %d" % (ns.mean(), ns.max()), "nt per model", np.bincount(w.obs_label.cpu().numpy()))
    print("total work %.3g quad-steps, per wave %.3g; heaviest pose %.3g (%.1fx a wave's share)" % (
        work.sum(), work.sum() / waves, work.max(), work.max() / (work.sum() / waves)))
    for k in order[:8]:
        print("  pose %d model %d iters %d ns %d nt %d work %.3g" % (k, w.pose_model[k].item(), it[k], ns[k], nt[k], work[k]))
    top = np.cumsum(work[order]) / work.sum()
    print("share of work in the heaviest 1%% / 5%% of poses: %.2f / %.2f" % (top[n // 100], top[n // 20]))


if __name__ == "__main__":
    main()
