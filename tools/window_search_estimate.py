#!/usr/bin/env python
"""Would an image-window correspondence search beat gicp_kernel's key scan?  Estimated on the CPU before building, on
C3-style candidates (tools/cycle_exit_sim.candidates) refined by the oracle's GICP with the cycle exit.

Every target t (an observed point, z > 0) lies on its pixel ray.  For a query q, d(q, t) >= dist(q, ray_t) =
|q x u_t| / |u_t| with u_t = (x/z, y/z, 1), and |q x u_t| >= q_z |a_t - a_q| (a = x/z), so
d(q, t) >= q_z |a_t - a_q| / c with c = max |u| over the segment (likewise in y).  Binning the targets into image cells
of `cell` pixels, a target whose cell is m >= 2 cells from the query's has |a_t - a_q| >= (m - 1) cell / fx, so an
upper bound B of the nearest distance (the previous iteration's correspondence, re-measured) limits the search to a
window of cells around the query's; the first strict minimum over the window's targets by (key, index) is the scan's.
Counted, per executed iteration and query: targets in the window (the keys to evaluate) and cells visited, against the
segment's targets (the scan's keys), overall and on the poses of >= 300 points; plus the share of wave passes (128
queries) whose every query has a window (q_z > 0, window within max_r cells) -- the others would scan.
    python tools/window_search_estimate.py [--per-object 8] [--out FILE.json]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-object", type=int, default=8)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--out")
    a = ap.parse_args()
    import cycle_exit_sim as S
    import oracle
    from perception_amd import synthetic as syn

    cam = syn.CAM_640
    fx, fy, cx, cy = cam["fx"], cam["fy"], cam["cx"], cam["cy"]
    res = {"cells": {}}
    for cell in (4, 8, 16):
        for max_r in (3, 6):
            key = f"cell{cell}_maxr{max_r}"
            acc = {"keys": 0, "scan_keys": 0, "cells": 0, "queries": 0, "passes": 0, "passes_windowed": 0,
                   "big_keys": 0, "big_scan": 0}
            res["cells"][key] = acc
    nposes = 0
    for src, scov, tgt, tcov in S.candidates(a.per_object, a.seed):
        src32 = src.astype(np.float32)
        tg = tgt.astype(np.float64)
        _, _, tr = oracle.gicp_trace(src32, scov, tgt.astype(np.float32), tcov, cycle_window=8)
        nposes += 1
        ns, nt = len(src), len(tg)
        at, bt = tg[:, 0] / tg[:, 2], tg[:, 1] / tg[:, 2]
        cmax = float(np.sqrt(1.0 + at ** 2 + bt ** 2).max())
        xs = [np.eye(4)]
        for r in tr:
            T = np.eye(4)
            T[:3, :3] = r[:9].reshape(3, 3)
            T[:3, 3] = r[9:12]
            xs.append(T)
        xs = xs[:len(tr)]
        prev = None
        for T in xs:
            R32 = T[:3, :3].astype(np.float32).astype(np.float64)
            t32 = T[:3, 3].astype(np.float32).astype(np.float64)
            q = src32.astype(np.float64) @ R32.T + t32
            d = ((q[:, None, :] - tg[None, :, :]) ** 2).sum(-1)
            nn = d.argmin(1)
            if prev is None:
                prev = nn
                for acc in res["cells"].values():  # the first iteration scans
                    acc["passes"] += (ns + 127) // 128
                    acc["keys"] += nt * ns
                    acc["scan_keys"] += nt * ns
                    if ns >= 300:
                        acc["big_keys"] += nt * ns
                        acc["big_scan"] += nt * ns
                continue
            B = np.sqrt(d[np.arange(ns), prev]) * 1.001 + 1e-6
            aq, bq = q[:, 0] / q[:, 2], q[:, 1] / q[:, 2]
            for cell in (4, 8, 16):
                ktx = np.rint((at * fx + cx) / cell).astype(np.int64)
                kty = np.rint((bt * fy + cy) / cell).astype(np.int64)
                kqx = np.rint((aq * fx + cx) / cell).astype(np.int64)
                kqy = np.rint((bq * fy + cy) / cell).astype(np.int64)
                # a target m cells away: |a_t - a_q| >= (m - 1) cell / f, so d >= q_z (m - 1) cell / (f c)
                rx = np.floor(1.0 + B * cmax * fx / (np.maximum(q[:, 2], 1e-9) * cell) + 0.01).astype(np.int64)
                ry = np.floor(1.0 + B * cmax * fy / (np.maximum(q[:, 2], 1e-9) * cell) + 0.01).astype(np.int64)
                inwin = (np.abs(ktx[None, :] - kqx[:, None]) <= rx[:, None]) & \
                        (np.abs(kty[None, :] - kqy[:, None]) <= ry[:, None])
                assert (inwin[np.arange(ns), nn]).all()  # the window holds the nearest target
                for max_r in (3, 6):
                    acc = res["cells"][f"cell{cell}_maxr{max_r}"]
                    ok = (q[:, 2] > 0) & (rx <= max_r) & (ry <= max_r)
                    for i0 in range(0, ns, 128):
                        sl = slice(i0, min(ns, i0 + 128))
                        acc["passes"] += 1
                        if ok[sl].all():
                            acc["passes_windowed"] += 1
                            k = int(inwin[sl].sum())
                            acc["cells"] += int(((2 * rx[sl] + 1) * (2 * ry[sl] + 1)).sum())
                        else:
                            k = nt * (sl.stop - sl.start)
                        acc["keys"] += k
                        acc["scan_keys"] += nt * (sl.stop - sl.start)
                        if ns >= 300:
                            acc["big_keys"] += k
                            acc["big_scan"] += nt * (sl.stop - sl.start)
                    acc["queries"] += ns
            prev = nn
    out = {"poses": nposes}
    for k, acc in res["cells"].items():
        out[k] = {"keys_vs_scan": acc["keys"] / max(acc["scan_keys"], 1),
                  "keys_vs_scan_ns_ge_300": acc["big_keys"] / max(acc["big_scan"], 1),
                  "cells_per_windowed_query": acc["cells"] / max(acc["queries"], 1),
                  "passes_windowed": acc["passes_windowed"] / max(acc["passes"], 1)}
    s_ = json.dumps(out, indent=1)
    print(s_)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s_ + "\n")


if __name__ == "__main__":
    main()
