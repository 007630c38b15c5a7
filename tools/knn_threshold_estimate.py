#!/usr/bin/env python
"""Would a threshold-prefiltered exact k-NN beat covariance_kernel's brute-force insertion scan?  (Round 6, the source
covariances are ~2 ms of a C3 step.)  Estimated on the CPU before building, on C3-style rendered clouds
(tests/helpers.SceneCase via tools/cycle_exit_sim.candidates, stride 8):
  the k = 10 neighbours of every point are the first k of all candidates by (distance, index); any threshold tau at or
  above the k-th smallest distance keeps them, so a scan that only collects candidates with d <= tau and sorts those
  is exact.  For thresholds taken from the sample grid around the point (the k-th smallest distance among its
  (2R+1)^2 grid neighbours; or the largest distance over a small fixed set) this counts the candidates per point such a
  scan collects, and their maximum per 64-point wave round (what a wave's insertion loop would run).
    python tools/knn_threshold_estimate.py [--per-object 60] [--out FILE.json]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402

K = 10


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-object", type=int, default=60)
    ap.add_argument("--out")
    a = ap.parse_args()
    import cycle_exit_sim as S
    from perception_amd import synthetic as syn
    cam, s = syn.CAM_640, 8
    clouds = [c[0].astype(np.float32) for c in S.candidates(a.per_object, 11)]
    variants = {"kth_of_5x5": ("kth", 2), "kth_of_7x7": ("kth", 3),
                "max_of_3x3_plus_axis4": ("max", [(x, y) for x in (-1, 0, 1) for y in (-1, 0, 1)] +
                                          [(2, 0), (-2, 0), (0, 2), (0, -2)])}
    res = {"clouds": 0, "brute_force_steps_per_point": None, "variants": {}}
    for name, (kind, arg) in variants.items():
        means, wave_max, npts, steps = [], [], 0, 0
        for P in clouds:
            n = len(P)
            if n <= K:
                continue
            kx = np.rint((P[:, 0] / P[:, 2] * cam["fx"] + cam["cx"]) / s).astype(int)
            ky = np.rint((P[:, 1] / P[:, 2] * cam["fy"] + cam["cy"]) / s).astype(int)
            grid = {(x, y): i for i, (x, y) in enumerate(zip(kx, ky))}
            d = ((P[:, None, :] - P[None, :, :]) ** 2).sum(-1)
            cnt = np.zeros(n, int)
            for i in range(n):
                if kind == "kth":
                    nb = [grid[(kx[i] + u, ky[i] + v)] for u in range(-arg, arg + 1) for v in range(-arg, arg + 1)
                          if (kx[i] + u, ky[i] + v) in grid]
                    tau = np.sort(d[i, nb])[K - 1] if len(nb) >= K else np.inf
                else:
                    nb = [grid[(kx[i] + u, ky[i] + v)] for u, v in arg if (kx[i] + u, ky[i] + v) in grid]
                    tau = d[i, nb].max() if len(nb) >= K else np.inf
                cnt[i] = int((d[i] <= tau).sum())
            means.append(cnt.mean())
            wave_max += [int(cnt[r:r + 64].max()) for r in range(0, n, 64)]
            npts += n
            steps += n * n
        res["clouds"] = len(means)
        res["brute_force_steps_per_point"] = steps / npts
        res["variants"][name] = {"collected_per_point": float(np.mean(means)),
                                 "wave_round_max_mean": float(np.mean(wave_max)),
                                 "wave_round_max_p90": float(np.percentile(wave_max, 90)),
                                 "threshold_steps_per_point": (2 * arg + 1) ** 2 - 1 if kind == "kth" else len(arg)}
    s_ = json.dumps(res, indent=1)
    print(s_)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s_ + "\n")


if __name__ == "__main__":
    main()
