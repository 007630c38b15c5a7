"""GICP covariances on the GPU (covariance_kernel through pcore_debug_covariances) bit for bit against the oracle's
restatement (orc_covariances: fast_gicp's k-nearest-neighbour covariance with PLANE regularisation, DESIGN.md section
5), on segments that exercise the k-NN list: random clouds, clouds on a lattice (many equal distances, so the
placement of ties decides the neighbour lists), duplicated points, fewer points than k, a single point, and a NaN point
among the first k candidates (the list that can no longer be sorted), a rendered-like plane patch and 256 / 257 points."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle  # noqa: E402
from perception_amd import _native  # noqa: E402

pytestmark = pytest.mark.gpu


def _segments():
    rng = np.random.default_rng(5)
    segs = []
    for n in (111, 467, 64, 65, 200):  # C3-like rendered clouds, tile boundaries
        segs.append((rng.normal(size=(n, 3)) * 0.05 + rng.normal(size=3)).astype(np.float32))
    g = np.stack(np.meshgrid(np.arange(7), np.arange(6), np.arange(3), indexing="ij"), -1).reshape(-1, 3)
    segs.append((g * 0.005 + np.array([0.1, -0.2, 0.9])).astype(np.float32))  # lattice: ties everywhere
    d = rng.normal(size=(40, 3)).astype(np.float32) * 0.01
    segs.append(np.concatenate([d, d[:20], d[5:9]]))  # duplicates
    segs.append(rng.normal(size=(7, 3)).astype(np.float32))  # n < k
    segs.append(rng.normal(size=(1, 3)).astype(np.float32))  # one point
    # a rendered-like patch (a tilted plane sampled on a pixel grid, unprojected: near-equal distances), 256 / 257 points
    u, v = np.meshgrid(np.arange(12) * 8.0, np.arange(10) * 8.0)
    z = 0.8 + 0.0005 * u + 0.0002 * v
    segs.append(np.stack([(u - 40) / 576.0 * z, (v - 30) / 576.0 * z, z], -1).reshape(-1, 3).astype(np.float32))
    segs.append((rng.normal(size=(256, 3)) * 0.05).astype(np.float32))
    segs.append((rng.normal(size=(257, 3)) * 0.05).astype(np.float32))
    nanseg = (rng.normal(size=(90, 3)) * 0.02).astype(np.float32)
    nanseg[3] = np.nan  # among the first k candidates of every point
    segs.append(nanseg)
    return segs


def _same(a, b):
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(np.where(na, 0.0, a).view(np.uint64),
                                                     np.where(nb, 0.0, b).view(np.uint64))


@pytest.mark.parametrize("k", [10, 5, 16])
def test_gpu_covariances_equal_oracle_bitwise(k):
    segs = _segments()
    cnt = np.array([len(s) for s in segs], np.int32)
    off = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.int32)
    xyz = np.concatenate(segs)
    xyzw = np.concatenate([xyz, np.zeros((len(xyz), 1), np.float32)], 1)
    dev = torch.device("cuda", 0)
    pts = torch.from_numpy(xyzw).to(dev)
    off_d, cnt_d = torch.from_numpy(off).to(dev), torch.from_numpy(cnt).to(dev)
    out = torch.full((len(xyz), 6), float("nan"), dtype=torch.float64, device=dev)
    lib = _native.load()
    assert lib.pcore_debug_covariances(pts.data_ptr(), off_d.data_ptr(), cnt_d.data_ptr(), len(segs), k,
                                       out.data_ptr(), None) == 0
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for s, o, c in zip(segs, off, cnt):
        want = oracle.covariances(s, k)
        assert _same(got[o:o + c], want), (len(s), k)


def _grid_clouds(cam_name="640"):
    """Clouds unprojected from a stride-8 sample grid of the camera (what render_cloud writes): tilted planes, a step
    (a depth discontinuity inside the neighbourhoods), 24 to 1,000 points -- the last one's window (40 x 25 cells) is
    larger than the kernel's LDS map, which sends it to the brute force."""
    from perception_amd import synthetic as syn
    cam, s = (syn.CAM_640 if cam_name == "640" else syn.CAM_1280), 8
    rng = np.random.default_rng(9)
    clouds = []
    for (w, h, x0, y0) in ((12, 10, 30, 20), (23, 20, 10, 5), (8, 3, 50, 40), (27, 17, 3, 30), (40, 25, 20, 10)):
        kx, ky = np.meshgrid(np.arange(x0, x0 + w), np.arange(y0, y0 + h))
        u, v = kx * s, ky * s
        z = 0.8 + 0.0004 * (u - cam["cx"]) + 0.0003 * (v - cam["cy"]) + rng.normal(size=u.shape) * 1e-3
        if w == 27:
            z = np.where(kx > x0 + 13, z + 0.05, z)  # a step: the far side's neighbourhoods reach across it
        z = np.round(z * 100) / 100  # the int-centimetre z-buffer's depths
        x = ((u.astype(np.float32) - np.float32(cam["cx"])) / np.float32(cam["fx"]) * z.astype(np.float32))
        y = ((v.astype(np.float32) - np.float32(cam["cy"])) / np.float32(cam["fy"]) * z.astype(np.float32))
        clouds.append(np.stack([x, y, z.astype(np.float32)], -1).reshape(-1, 3).astype(np.float32))
    return clouds, cam, s


@pytest.mark.parametrize("cam_name", ["640", "1280"])
def test_gpu_threshold_knn_covariances_equal_oracle_bitwise(cam_name):
    """covariance_cloud_kernel (the threshold k-NN over each rendered cloud's sample grid, pcore_cov.h; k = 10) bit for
    bit against the oracle: on grid-structured clouds (the path it serves) and on every segment of the brute-force test
    (no grid structure, lattices with ties, duplicates, n < k, a NaN point: the threshold stays a valid bound or the
    kernel falls back), each in a slot of a strided buffer as the ICP scratch holds them."""
    grid, cam, s = _grid_clouds(cam_name)
    # clustered clouds in front of the camera that share few sample-grid cells: the map keeps one point per cell, so the
    # neighbourhood bound is loose or infinite and the lists overflow -- a cloud small enough for the LDS copy (the
    # brute force then overwrites the copy with its tile) and a larger one
    rng = np.random.default_rng(21)
    clustered = [np.stack([rng.normal(size=n) * 0.002, rng.normal(size=n) * 0.002, 0.8 + rng.random(n) * 0.1], -1)
                 .astype(np.float32) for n in (50, 90)]
    segs = grid + clustered + _segments()
    cap = max(len(x) for x in segs)
    xyzw = np.zeros((len(segs) * cap, 4), np.float32)
    for i, x in enumerate(segs):
        xyzw[i * cap:i * cap + len(x), :3] = x
    cnt = np.array([len(x) for x in segs], np.int32)
    dev = torch.device("cuda", 0)
    pts = torch.from_numpy(xyzw).to(dev)
    cnt_d = torch.from_numpy(cnt).to(dev)
    out = torch.full((len(segs) * cap, 6), float("nan"), dtype=torch.float64, device=dev)
    lib = _native.load()
    assert lib.pcore_debug_covariances_cloud(pts.data_ptr(), cnt_d.data_ptr(), cap, len(segs), cam["fx"], cam["fy"],
                                             cam["cx"], cam["cy"], s, out.data_ptr(), None) == 0
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for i, x in enumerate(segs):
        assert _same(got[i * cap:i * cap + len(x)], oracle.covariances(x, 10)), (i, len(x))
