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
