"""GPU: the recognizer's per-state work on the device (pcore_state_poses, pcore_count_within) against the host
restatements it replaces -- bit for bit.

  pcore_state_poses   vs ObjectRecognizer._pose_in_cam's arithmetic (model.quat_xyzw_to_matrix_batch,
                      pose_matrix_batch, chain_matmul_batch, init_from_eigen_batch): GetStateImagesUnifiedGPU's
                      pose building (search_env.cpp:1535-1576);
  pcore_count_within  vs a numpy float32 loop of PCL's radiusSearch count (IsValidPose, search_env.cpp:359-396),
                      the restatement tests/test_valid_pose.py pins on the CPU.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from perception_amd import synthetic as syn
from perception_amd.core import PoseCore
from perception_amd.model import chain_matmul_batch, compute_proj, init_from_eigen_batch, pose_matrix_batch
from tests.test_valid_pose import _pcl_counts

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _core():
    cam = syn.CAM_640
    core = PoseCore(0)
    core.set_camera(cam["width"], cam["height"], cam["fx"], cam["fy"], cam["cx"], cam["cy"],
                    compute_proj(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["width"], cam["height"]))
    return core


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def test_state_poses_bit_exact_vs_host_chain():
    rng = np.random.default_rng(11)
    n, K = 20000, 5
    states = np.empty((n, 7))
    states[:, :3] = rng.normal(scale=0.4, size=(n, 3)) + np.array([0.0, 0.0, 0.9])
    states[:, 3:] = rng.normal(size=(n, 4)) * rng.uniform(0.2, 3.0, size=(n, 1))  # not normalised
    states[:7, 3:] = [[0, 0, 0, 1], [1, 0, 0, 0], [0, 0, 0, -1], [0.5, 0.5, 0.5, 0.5], [0, 0, 1e-8, 1],
                      [0, 0, 0, 1e-30], [-0.0, 0.0, -0.0, 1.0]]
    model = rng.integers(0, K, n).astype(np.int32)
    pre = np.stack([np.eye(4) for _ in range(K)])
    for k in range(K):
        pre[k, :3, 3] = rng.normal(scale=0.05, size=3)
        pre[k, 2, 2] = -1.0 if k == 3 else 1.0
        pre[k] = pre[k].astype(np.float32).astype(np.float64)
    cam_pose = np.eye(4)
    cam_pose[:3, :3] = pose_matrix_batch(np.zeros((1, 3)), rng.normal(size=(1, 4)))[0, :3, :3]
    cam_pose[:3, 3] = rng.normal(size=3)
    cam_matrix = np.linalg.inv(cam_pose)
    want = init_from_eigen_batch(chain_matmul_batch(cam_matrix, pose_matrix_batch(states[:, :3], states[:, 3:7]),
                                                    pre[model]), 100)
    core = _core()
    got = core.state_poses(torch.from_numpy(states).to(DEV), torch.from_numpy(model).to(DEV), cam_matrix,
                           torch.from_numpy(pre.reshape(K, 16)).to(DEV)).cpu().numpy()
    assert np.array_equal(_bits(got), _bits(want))
    # empty batch
    out = core.state_poses(torch.zeros((0, 7), dtype=torch.float64, device=DEV),
                           torch.zeros(0, dtype=torch.int32, device=DEV), cam_matrix,
                           torch.from_numpy(pre.reshape(K, 16)).to(DEV))
    assert out.shape == (0, 16)


def test_count_within_matches_pcl_restatement():
    rng = np.random.default_rng(12)
    cam = syn.CAM_640
    core = _core()
    # an observation with three labelled segments (plus unlabelled points), as set_observation takes it
    pts, labs = [], []
    for L, c in enumerate([(-0.1, 0.0, 0.8), (0.05, 0.02, 0.9), (0.15, -0.05, 0.7)]):
        m = 80 + 60 * L
        pts.append(np.asarray(c) + rng.normal(scale=0.03, size=(m, 3)))
        labs.append(np.full(m, L, np.int32))
    pts.append(rng.normal(scale=0.2, size=(50, 3)) + np.array([0, 0, 1.0]))
    labs.append(np.full(50, -1, np.int32))
    xyz = np.concatenate(pts).astype(np.float32)
    lab = np.concatenate(labs)
    perm = rng.permutation(len(xyz))
    xyz, lab = xyz[perm], lab[perm]
    H, W = cam["height"], cam["width"]
    mask = np.zeros((H, W), np.uint8)
    mask[0, :3] = [1, 2, 3]  # labels 0..2 present in the mask
    core.set_observation(torch.zeros((H, W), dtype=torch.int32, device=DEV), torch.from_numpy(mask).to(DEV),
                         torch.from_numpy(xyz).to(DEV), torch.from_numpy(lab).to(DEV), 0.01)
    n = 3000
    ql = rng.integers(-1, 5, n).astype(np.int32)  # labels outside the segments count 0
    centres = np.array([(-0.1, 0.0, 0.8), (0.05, 0.02, 0.9), (0.15, -0.05, 0.7), (0, 0, 1), (0, 0, 1), (0, 0, 1)])
    q = centres[np.clip(ql, 0, 5)] + rng.normal(scale=0.05, size=(n, 3))
    radius = rng.choice([0.02, 0.0566, 0.11], n)
    r2 = (radius * radius).astype(np.float32)
    got = core.count_within(torch.from_numpy(q.astype(np.float32)).to(DEV), torch.from_numpy(ql).to(DEV),
                            torch.from_numpy(r2).to(DEV)).cpu().numpy()
    want = np.zeros(n, np.int64)
    for L in range(3):
        seg = xyz[lab == L]
        for r in np.unique(radius):
            sel = (ql == L) & (radius == r)
            if sel.any():
                want[sel] = _pcl_counts(q[sel], seg, r)
    assert np.array_equal(got, want)
    assert got[(ql < 0) | (ql > 2)].sum() == 0
