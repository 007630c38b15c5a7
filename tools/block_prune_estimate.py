#!/usr/bin/env python
"""Would skipping blocks of target quads in gicp_kernel's correspondence scan pay?  (Round 6: the search is 71 % of an
iteration on the heavy chains that end the launch, profiles/r06j/gicp_phase_profbig.txt.)  Estimated on the CPU before
building, on C3-style candidates (tools/cycle_exit_sim.candidates: rendered clouds against their label's observed
segment, stride 8) refined by the oracle's GICP with the cycle exit (its executed iterations).

The scan stays exact if it skips a block of consecutive targets (in segment order, so the first-strict-minimum
tie-break by index is untouched) whose bounding box is farther from every query of the wave's pass (the 128 source
points a pass pairs up) than an upper bound B of that query's nearest distance: every skipped target is then strictly
worse than the minimum.  B here is the distance to the query's previous-iteration correspondence (the first iteration
scans everything) and, in the "running" variant, also the best distance of the blocks scanned so far.  "union" tests
each block's box against one wave-uniform box, the union of the pass's query boxes [q - sqrt(B), q + sqrt(B)] (a
scalar test per block instead of a per-lane one).  Counted: the
fraction of (query, target) steps still scanned, overall and on the poses of >= 300 points, per block size.
    python tools/block_prune_estimate.py [--per-object 8] [--out FILE.json]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402


def boxes(tgt, bsz):
    n = len(tgt)
    lo = np.array([tgt[i:i + bsz].min(0) for i in range(0, n, bsz)])
    hi = np.array([tgt[i:i + bsz].max(0) for i in range(0, n, bsz)])
    return lo, hi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-object", type=int, default=8)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--out")
    a = ap.parse_args()
    import cycle_exit_sim as S
    import oracle

    sizes = (16, 32, 64)
    VAR = ("prev", "running", "union")
    tot = {v: {b: [0, 0] for b in sizes} for v in VAR}
    big = {v: {b: [0, 0] for b in sizes} for v in VAR}
    nposes = iters_total = 0
    for src, scov, tgt, tcov in S.candidates(a.per_object, a.seed):
        tgt = tgt.astype(np.float64)
        src32 = src.astype(np.float32)
        _, _, tr = oracle.gicp_trace(src32, scov, tgt.astype(np.float32), tcov, cycle_window=8)
        nposes += 1
        ns, nt = len(src), len(tgt)
        bx = {b: boxes(tgt, b) for b in sizes}
        xs = [np.eye(4)]
        for r in tr:
            T = np.eye(4)
            T[:3, :3] = r[:9].reshape(3, 3)
            T[:3, 3] = r[9:12]
            xs.append(T)
        xs = xs[:len(tr)]  # the transform at the top of each executed iteration
        iters_total += len(xs)
        prev = None
        for T in xs:
            R32 = T[:3, :3].astype(np.float32).astype(np.float64)
            t32 = T[:3, 3].astype(np.float32).astype(np.float64)
            q = src32.astype(np.float64) @ R32.T + t32
            d = ((q[:, None, :] - tgt[None, :, :]) ** 2).sum(-1)
            nn = d.argmin(1)
            B = d[np.arange(ns), prev] if prev is not None else np.full(ns, np.inf)
            for b in sizes:
                lo, hi = bx[b]
                gap = np.maximum(np.maximum(lo[None] - q[:, None], q[:, None] - hi[None]), 0.0)
                lb = (gap ** 2).sum(-1)  # (ns, nblocks)
                nb = lo.shape[0]
                bsz_t = np.array([min(b, nt - k * b) for k in range(nb)])
                for i0 in range(0, ns, 128):
                    sl = slice(i0, min(ns, i0 + 128))
                    full = nt * 128  # the pass's lanes x targets (a one-query pass still takes the lanes)
                    need = (lb[sl] <= B[sl, None]).any(0)
                    sc_prev = int(bsz_t[need].sum()) * 128
                    # running: blocks in order; B tightens with the scanned blocks' minimum
                    Bq = B[sl].copy()
                    sc_run = 0
                    for k in range(nb):
                        if (lb[sl, k] <= Bq).any():
                            sc_run += int(bsz_t[k]) * 128
                            Bq = np.minimum(Bq, d[sl, k * b:k * b + bsz_t[k]].min(1))
                    # union: one wave-uniform box, the pass's queries' boxes [q - sqrt(B), q + sqrt(B)] merged
                    sB = np.sqrt(B[sl])[:, None]
                    ulo, uhi = (q[sl] - sB).min(0), (q[sl] + sB).max(0)
                    hit = ((lo <= uhi[None]) & (hi >= ulo[None])).all(1)
                    sc_uni = int(bsz_t[hit].sum()) * 128
                    for v, sc in (("prev", sc_prev), ("running", sc_run), ("union", sc_uni)):
                        tot[v][b][0] += sc
                        tot[v][b][1] += full
                        if ns >= 300:
                            big[v][b][0] += sc
                            big[v][b][1] += full
            prev = nn
    res = {"poses": nposes, "executed_iterations": iters_total, "block_targets": list(sizes),
           "scanned_fraction": {v: {str(b): tot[v][b][0] / max(tot[v][b][1], 1) for b in sizes} for v in tot},
           "scanned_fraction_ns_ge_300": {v: {str(b): big[v][b][0] / max(big[v][b][1], 1) for b in sizes} for v in big}}
    s_ = json.dumps(res, indent=1)
    print(s_)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s_ + "\n")


if __name__ == "__main__":
    main()
