"""GPU: ADD / ADD-S (pcore_pose_distances) against the reference's pose_error golden and the f64 oracle.
Tolerance 1e-12 m: both sides are f64; only the summation order differs."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle
from perception_amd import metrics
from perception_amd.core import PoseCore

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def core():
    return PoseCore(0)


def test_add_adi_match_reference_pose_error_golden(core):
    g = np.load(os.path.join(G, "pose_error.npz"))
    pts = g["pts"].astype(np.float32)
    for m in range(len(g["add"])):
        # the golden points are f64; f32 model points (as from a PLY) move the result by < 1e-8 m
        a = metrics.add(core, g["R_est"][m], g["t_est"][m], g["R_gt"][m], g["t_gt"][m], pts)
        s = metrics.adi(core, g["R_est"][m], g["t_est"][m], g["R_gt"][m], g["t_gt"][m], pts)
        assert abs(a - g["add"][m]) < 1e-7
        assert abs(s - g["adi"][m]) < 1e-7


@pytest.mark.parametrize("n", [1, 255, 256, 1025, 3000])
def test_pose_distances_match_oracle(core, n):
    rng = np.random.default_rng(n)
    pts = rng.uniform(-0.1, 0.1, (n, 3)).astype(np.float32)
    M = 7
    Tg = np.tile(np.eye(4), (M, 1, 1))
    Te = np.tile(np.eye(4), (M, 1, 1))
    for m in range(M):
        Tg[m, :3, :3] = np.linalg.qr(rng.normal(size=(3, 3)))[0]
        Tg[m, :3, 3] = rng.uniform(-0.3, 0.3, 3) + [0, 0, 0.8]
        Te[m, :3, :3] = Tg[m, :3, :3] @ np.linalg.qr(np.eye(3) + 0.05 * m * rng.normal(size=(3, 3)))[0]
        Te[m, :3, 3] = Tg[m, :3, 3] + rng.normal(0, 0.005 * m, 3)
    add, adds = metrics.pose_distances(core, pts, Tg, Te)
    oadd, oadds = oracle.pose_distances(pts, Tg, Te)
    assert np.allclose(add.cpu().numpy(), oadd, rtol=0, atol=1e-12)
    assert np.allclose(adds.cpu().numpy(), oadds, rtol=0, atol=1e-12)
    assert adds.cpu().numpy()[0] <= add.cpu().numpy()[0] + 1e-15


def test_pose_distances_rejects_empty_model(core):
    with pytest.raises(Exception):
        metrics.pose_distances(core, np.zeros((0, 3), np.float32), np.eye(4)[None], np.eye(4)[None])
