#!/usr/bin/env python
"""Would a tile-first raster order beat the fused kernel's triangle-first stream walk?  (estimate
before building; build only for a predicted >= 15 % fewer VALU per pose.)

Tile-first: the sample grid is cut into t x t tiles of samples; every triangle whose sample window (the kernel's
per-triangle window, image_renderer.cuh:86-111 at stride s) touches samples is binned into the tiles it overlaps;
then each tile is rastered with one lane per sample, one wave step per binned triangle (t = 8: a tile is one wave;
t = 4 / 2: 4 / 16 tiles share a wave step).  Under the a6' contract every fragment still takes part in the min, so
the binned pairs are the work unless a tile can prove a triangle hidden (Hi-Z), which round 4 bounded by 3.5-9.5 %
of the triangles (tools/cull_estimate.py).

Counted here on C2-style poses (tests/helpers.SceneCase, the 003_cracker_box proxy, stride 8), from the poses'
projected vertices (numpy, no GPU):
  fragment_tests   sum over triangles of the samples in their window (the triangle-first scheme's fragment tests),
  pairs[t]         (triangle, tile) pairs a tile-first binning creates,
and priced with the fused kernel's measured per-stage VALU (profiles/r05y/fused_valu_ablation.txt, per pose of C2):
vertex stage 5.0 k, triangle windows 5.9 k, record flush (fragment tests) 5.5 k, phase 2 + the rest 3.9 k.  A
tile-first kernel keeps the vertex stage, the triangle windows (binning needs them) and phase 2, adds the binning
(>= 4 wave-VALU per 64 appended pairs: the append address, the store, the count) and replaces the flush with
pairs[t] * t^2 lane-tests at the flush's own measured price per 64 lane-tests (5.5 k VALU / (fragment tests / 64):
the same barycentric, inside-test, certified-depth and LDS-min arithmetic per lane, whichever order feeds it).  The
triangle-first flush packs one lane per (triangle, sample) record, so it already runs at one lane-test per fragment
test; a tile of t x t samples spends t^2 lane-tests on every (triangle, tile) pair.
    python tools/tile_first_estimate.py [--poses 200] [--out FILE.json]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

VALU = {"vertex": 5.0e3, "triangle_windows": 5.9e3, "flush": 5.5e3, "phase2_rest": 3.9e3}  # r05y, per C2 pose
C_BIN = 4.0     # wave-VALU per 64 appended (triangle, tile) pairs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--poses", type=int, default=200)
    ap.add_argument("--stride", type=int, default=8)
    ap.add_argument("--out")
    a = ap.parse_args()
    from tests.helpers import SceneCase

    case = SceneCase(("003_cracker_box",), n_poses=a.poses)
    sc = case.scene
    W, H, s = sc.width, sc.height, a.stride
    tris = sc.bank.tris.reshape(-1, 3, 3).astype(np.float64)
    P = np.asarray(sc.proj, np.float64).reshape(4, 4)
    nx, ny = W // s, (H + s - 1) // s
    tiles = (8, 4, 2)
    frag = hit = 0
    pairs = {t: 0 for t in tiles}
    npose = 0
    for i in range(len(case.poses)):
        m = case.poses[i].astype(np.float64).reshape(4, 4)
        cam = tris @ m[:3, :3].T + m[:3, 3]
        z = cam[..., 2]
        if z.min() <= 1:
            continue
        npose += 1
        sx = (cam @ P[0, :3] + P[0, 3]) / z * W / 2 + W / 2
        sy = (cam @ P[1, :3] + P[1, 3]) / z * H / 2 + H / 2
        x0, x1 = np.clip(sx.min(1), 0, W - 1), np.clip(sx.max(1), 0, W - 1)
        y0, y1 = np.clip(sy.min(1), 0, H - 1), np.clip(sy.max(1), 0, H - 1)
        kx0, kx1 = np.maximum(0, np.ceil(x0 / s)), np.minimum(nx - 1, np.floor(x1 / s))
        r0, r1 = H - 1 - y1, H - 1 - y0  # image rows (the reference writes row H - 1 - y)
        ky0, ky1 = np.maximum(0, np.ceil(r0 / s)), np.minimum(ny - 1, np.floor(r1 / s))
        ok = (kx1 >= kx0) & (ky1 >= ky0)
        hit += int(ok.sum())
        frag += int(((kx1 - kx0 + 1) * (ky1 - ky0 + 1))[ok].sum())
        for t in tiles:
            tx = np.floor(kx1[ok] / t) - np.floor(kx0[ok] / t) + 1
            ty = np.floor(ky1[ok] / t) - np.floor(ky0[ok] / t) + 1
            pairs[t] += int((tx * ty).sum())
    res = {"poses": npose, "triangles": len(tris), "stride": s,
           "triangles_touching_samples_per_pose": hit / npose, "fragment_tests_per_pose": frag / npose,
           "triangle_first_valu_per_pose": sum(VALU.values()), "tile_first": {}}
    c_step = VALU["flush"] / (frag / npose / 64.0)  # measured wave-VALU per 64 lane-tests of the flush
    res["flush_valu_per_64_lane_tests"] = c_step
    for t in tiles:
        pp = pairs[t] / npose
        raster = pp * t * t / 64.0 * c_step
        binning = pp / 64 * C_BIN
        total = VALU["vertex"] + VALU["triangle_windows"] + VALU["phase2_rest"] + binning + raster
        res["tile_first"][f"{t}x{t}"] = {
            "pairs_per_pose": pp, "raster_valu": raster, "binning_valu": binning, "valu_per_pose": total,
            "vs_triangle_first": total / res["triangle_first_valu_per_pose"] - 1.0,
            "with_ideal_9.5pct_culling": (total - 0.095 * (raster + binning)) / res["triangle_first_valu_per_pose"] - 1.0}
    best = min(v["with_ideal_9.5pct_culling"] for v in res["tile_first"].values())
    res["build"] = bool(best <= -0.15)
    res["build_threshold"] = -0.15
    s_ = json.dumps(res, indent=1)
    print(s_)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s_ + "\n")


if __name__ == "__main__":
    main()
