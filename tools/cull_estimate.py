import sys, numpy as np
sys.path.insert(0, '/root/repo')
import oracle
from tests.helpers import SceneCase
from scipy.cluster.vq import kmeans2
case = SceneCase(("003_cracker_box",), n_poses=300)
sc = case.scene
tris = sc.bank.tris.reshape(-1, 3, 3).astype(np.float64)
n = len(case.poses)
W, H, s = sc.width, sc.height, 8
src = np.full((H, W), 2**31 - 1, np.int32)
depth = oracle.render_depth(sc.bank.tris, sc.bank.tris_model_count, case.poses, np.zeros(n, np.int32),
                            np.zeros(n, np.int32), W, H, sc.proj, src, np.zeros((H, W), np.uint8), 1.0)
P = np.asarray(sc.proj, np.float64).reshape(4, 4)
cent = tris.mean(1)
for K in (8, 16, 24, 32, 48):
    _, lab = kmeans2(cent, K, seed=1, minit='++')
    culled = 0.0
    for i in range(n):
        m = case.poses[i].astype(np.float64).reshape(4, 4)
        zs = depth[i, ::s, ::s]  # sample (ky, kx)
        for k in range(K):
            v = tris[lab == k].reshape(-1, 3)
            if len(v) == 0: continue
            lo, hi = v.min(0), v.max(0)
            c = np.array([[x, y, z] for x in (lo[0], hi[0]) for y in (lo[1], hi[1]) for z in (lo[2], hi[2])])
            cam = c @ m[:3, :3].T + m[:3, 3]
            lz = cam[:, 2]
            if lz.min() <= 1: continue
            px = cam @ P[0, :3] + P[0, 3]; py = cam @ P[1, :3] + P[1, 3]
            sx = px / lz * W / 2 + W / 2; sy = py / lz * H / 2 + H / 2
            x0, x1 = sx.min() - 2, sx.max() + 2; y0, y1 = sy.min() - 2, sy.max() + 2
            # image row = H-1-sy
            kx0, kx1 = max(0, int(np.ceil(x0 / s))), min(W // s - 1, int(np.floor(x1 / s)))
            r0, r1 = H - 1 - y1, H - 1 - y0
            ky0, ky1 = max(0, int(np.ceil(r0 / s))), min((H + s - 1) // s - 1, int(np.floor(r1 / s)))
            if kx1 < kx0 or ky1 < ky0:
                culled += (lab == k).sum(); continue
            win = zs[ky0:ky1 + 1, kx0:kx1 + 1]
            zb = np.floor(lz.min() * (1 - 1e-5) + 0.5)
            if np.all((win > 0) & (win <= zb)):
                culled += (lab == k).sum()
    print(K, "culled triangle fraction (final z, best case): %.3f" % (culled / (n * len(tris))), flush=True)
