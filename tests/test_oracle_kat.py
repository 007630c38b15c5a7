"""Analytic known-answer tests of the CPU oracle (SURVEY.md 8c "Known-answer tests").  These pin the
restatement where no reference golden vector exists (parity vs the reference binary is unpinned)."""
import numpy as np
import pytest

import oracle
from perception_amd.model import compute_proj, init_from_eigen_batch

W, H = 64, 48
FX = FY = 60.0
CX, CY = 31.5, 23.5


def _proj():
    return oracle.compute_proj(FX, FY, CX, CY, W, H)


def _pose(t=(0.0, 0.0, 0.8)):
    T = np.eye(4)
    T[:3, 3] = t
    return init_from_eigen_batch(T[None])


def _square(half=0.1, z=0.0):
    a, b, c, d = (-half, -half, z), (half, -half, z), (half, half, z), (-half, half, z)
    return np.array([a + b + c, a + c + d], np.float32)


def _render(tris, poses, src=None, mask=None, labels=None, thr=1.0, proj=None, w=W, h=H):
    n = len(poses)
    src = np.zeros((h, w), np.int32) if src is None else src
    return oracle.render_depth(tris, [len(tris)], poses, np.zeros(n, np.int32), labels, w, h,
                               _proj() if proj is None else proj, src, mask, thr)


def test_compute_proj_host_mirror_is_bitwise_equal():
    for args in ((576.09757860, 576.09757860, 321.06398107, 242.97676897, 640, 480),
                 (1152.195, 1152.195, 640.0, 360.0, 1280, 720), (FX, FY, CX, CY, W, H)):
        assert np.array_equal(oracle.compute_proj(*args, 10.0, 10000.0).view(np.uint32),
                              compute_proj(*args).view(np.uint32))


def test_fronto_parallel_square_depth_is_80cm():
    z = _render(_square(), _pose())[0]
    covered = z > 0
    assert covered.sum() > 50
    assert set(np.unique(z[covered])) == {80}
    # the square spans +-0.1 m at 0.8 m: about 2 * 0.1 / 0.8 * 60 = 15 px wide
    cols = np.nonzero(covered.any(0))[0]
    assert 13 <= len(cols) <= 17


def test_empty_and_behind_camera():
    assert _render(_square(), _pose((0, 0, -0.8)))[0].max() <= 0
    assert _render(_square(), _pose((5.0, 0, 0.8)))[0].max() == 0


def test_unprojection_of_a_known_pixel():
    d = np.zeros((H, W), np.int32)
    d[24, 16] = 100
    xyz, pose, lab = oracle.depth_to_cloud(d, 8, CX, CY, FX, FY, 100.0)
    assert xyz.shape == (1, 3)
    z = np.float32(100) / np.float32(100.0)
    assert np.array_equal(xyz[0], np.array([(np.float32(16) - np.float32(CX)) / np.float32(FX) * z,
                                            (np.float32(24) - np.float32(CY)) / np.float32(FY) * z, z], np.float32))
    d[25, 16] = 50  # not on the stride grid -> ignored
    assert oracle.depth_to_cloud(d, 8, CX, CY, FX, FY, 100.0)[0].shape == (1, 3)


def test_cloud_order_is_pose_row_col_and_labels():
    d = np.zeros((2, H, W), np.int32)
    d[0, 8, 40] = 10
    d[0, 0, 8] = 20
    d[1, 0, 0] = 30
    xyz, pose, lab = oracle.depth_to_cloud(d, 8, CX, CY, FX, FY, 100.0, pose_label=np.array([4, 7], np.int32))
    assert list(pose) == [0, 0, 1]
    assert list(np.round(xyz[:, 2] * 100).astype(int)) == [20, 10, 30]
    assert list(lab) == [4, 4, 7]
    m = np.zeros((H, W), np.uint8)
    m[0, 8] = 3
    xyz, pose, lab = oracle.depth_to_cloud(d[0], 8, CX, CY, FX, FY, 100.0, label_mask=m)
    assert len(xyz) == 1 and lab[0] == 2


def _eval(tris, poses, obs_xyz, tot, labels=True, src=None, mask=None):
    n = len(poses)
    src = np.zeros((H, W), np.int32) if src is None else src
    mask = np.ones((H, W), np.uint8) if (mask is None and labels) else mask
    return oracle.evaluate(tris, [len(tris)], poses, np.zeros(n, np.int32), np.zeros(n, np.int32) if labels else None,
                           W, H, _proj(), src, mask, 1.0, 4, CX, CY, FX, FY, 100.0, obs_xyz,
                           np.array([0], np.int32) if labels else None,
                           np.array([len(obs_xyz)], np.int32) if labels else None,
                           np.full(n, tot, np.float32), 2 if labels else 0, True, 0.01)


def test_identical_render_and_observation_costs_zero():
    tris, poses = _square(), _pose()
    z = _render(tris, poses)
    xyz, _, _ = oracle.depth_to_cloud(z, 4, CX, CY, FX, FY, 100.0)
    rc, oc, df = _eval(tris, poses, xyz, len(xyz))
    assert rc[0] == 0.0 and oc[0] == 0.0 and df[0] == 0.0


def test_far_observation_is_all_bad_and_no_points_is_invalid():
    tris, poses = _square(), _pose()
    far = np.array([[0.0, 0.0, 5.0]], np.float32)
    rc, oc, df = _eval(tris, poses, far, 1)
    assert rc[0] == 100.0 and oc[0] == 100.0
    rc, oc, df = _eval(tris, _pose((5.0, 0, 0.8)), far, 1)
    assert rc[0] == -1.0  # cost_percentage_functor: no rendered points


def test_source_occlusion_3dof_threshold():
    tris, poses = _square(), _pose()
    clear = _render(tris, poses)[0]
    src = np.zeros((H, W), np.int32)
    src[clear > 0] = 78   # 2 cm in front of the render: occludes (> 1 cm)
    z = _render(tris, poses, src=src, thr=1.0)[0]
    assert z.max() == 0
    src[clear > 0] = 79   # exactly 1 cm: |80 - 79| > 1.0 is false -> kept
    assert np.array_equal(_render(tris, poses, src=src, thr=1.0)[0], clear)
    src[clear > 0] = 85   # source behind the render: kept
    assert np.array_equal(_render(tris, poses, src=src, thr=1.0)[0], clear)


def test_source_occlusion_6dof_labels():
    tris, poses = _square(), _pose()
    clear = _render(tris, poses)[0]
    src = np.zeros((H, W), np.int32)
    src[clear > 0] = 79
    mask = np.zeros((H, W), np.uint8)
    mask[clear > 0] = 2   # another object's label (pose label 0 <-> mask 1)
    z = _render(tris, poses, src=src, mask=mask, labels=np.zeros(1, np.int32))[0]
    assert z.max() == 0
    mask[clear > 0] = 1   # same object: never occluded by itself
    z = _render(tris, poses, src=src, mask=mask, labels=np.zeros(1, np.int32))[0]
    assert np.array_equal(z, clear)


def test_nearer_triangle_wins_regardless_of_order():
    near, far = _square(0.05, 0.0), _square(0.1, 0.1)  # model z +0.1 -> 10 cm further
    a = _render(np.concatenate([near, far]), _pose())[0]
    b = _render(np.concatenate([far, near]), _pose())[0]
    assert np.array_equal(a, b)
    assert set(np.unique(a[a > 0])) == {80, 90}


def test_degenerate_triangle_nan_fragments_write_depth_zero():
    # proj with x/y rows = identity: a triangle at camera y = 0 projects onto screen row H/2 exactly,
    # its area is exactly 0, and pixels on that row get NaN barycentrics (inside) -> int32(NaN) = 0.
    proj = np.zeros(16, np.float32)
    proj[0] = 1.0
    proj[5] = 1.0
    proj[10] = 1.0
    proj[14] = 1.0
    line = np.array([[-0.3, 0.0, 0.0, 0.0, 0.0, 0.0, 0.3, 0.0, 0.0]], np.float32)
    behind = _square(0.9, 0.2)  # a big quad 20 cm behind
    z = _render(np.concatenate([behind, line]), _pose(), proj=proj)[0]
    ref = _render(behind, _pose(), proj=proj)[0]
    row = H - 1 - H // 2
    assert (ref[row] > 0).any()
    diff = np.nonzero(z != ref)
    assert set(diff[0]) == {row}      # only the degenerate row changed ...
    assert (z[diff] == 0).all()       # ... to depth 0


def test_select_semantics():
    rc = np.array([5, 3, 3, -1, 3, 90, 10, 10], np.float32)
    oc = np.array([5, 4, 4, 0, 4, 10, 50, 0.5], np.float32)
    pm = np.array([0, 0, 0, 0, 1, 1, 2, 2], np.int32)
    cost, idx = oracle.select(rc, oc, pm, 4, index_base=100)
    assert list(cost[:3]) == [7, 7, 10]
    assert list(idx[:3]) == [101, 104, 107]   # ties: lowest index; |10 - 50| >= 30 filtered
    assert cost[3] == 2**31 - 1 and idx[3] == -1


def test_knn_ties_pick_lowest_index():
    o = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0]], np.float32)
    d2, idx = oracle.knn1(np.zeros((1, 3), np.float32), None, o)
    assert idx[0] == 0 and d2[0] == 1.0
    d2, idx = oracle.knn1(np.zeros((1, 3), np.float32), np.array([1], np.int32), o,
                          np.array([0, 1], np.int32), np.array([1, 3], np.int32))
    assert idx[0] == 1
    d2, idx = oracle.knn1(np.zeros((1, 3), np.float32), np.array([5], np.int32), o,
                          np.array([0], np.int32), np.array([3], np.int32))
    assert idx[0] == -1 and np.isinf(d2[0])


def _box_cloud(n=300, seed=0):
    from perception_amd import synthetic as syn
    rng = np.random.default_rng(seed)
    m = syn.ycb_proxy("003_cracker_box", 8)
    pts = np.unique(m.tris.reshape(-1, 3), axis=0).astype(np.float32) + np.float32([0.05, -0.02, 0.8])
    return pts[rng.choice(len(pts), n, replace=False)]


@pytest.mark.parametrize("offset", [(0.01, -0.005, 0.008), (-0.004, 0.012, -0.006)])
def test_gicp_recovers_a_translation(offset):
    """GICP spec (correspondences by the three-FMA key): a cloud shifted by a centimetre-scale
    offset is registered back onto itself -- T's translation is minus the offset, its rotation the identity."""
    tgt = _box_cloud()
    src = tgt + np.float32(offset)
    T, it = oracle.gicp(src, oracle.covariances(src), tgt, oracle.covariances(tgt))
    assert 1 <= it < 150
    assert np.allclose(T[:3, 3], -np.asarray(offset), atol=1e-5)
    assert np.abs(T[:3, :3] - np.eye(3)).max() < 1e-5


def test_gicp_recovers_a_small_rigid_motion():
    """A 3-degree rotation about the cloud's centre plus a 5 mm shift is undone to within 1e-4."""
    tgt = _box_cloud(seed=1)
    c = tgt.mean(0)
    a = np.deg2rad(3.0)
    Rz = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
    src = ((tgt - c) @ Rz.T + c + np.array([0.005, 0.0, -0.003])).astype(np.float32)
    T, it = oracle.gicp(src, oracle.covariances(src), tgt, oracle.covariances(tgt))
    back = src.astype(np.float64) @ T[:3, :3].T + T[:3, 3]
    assert it < 150
    assert np.abs(back - tgt).max() < 1e-4


def test_render_color_nearest_triangle_and_black_out():
    """Colour planes of the oracle's serial z-test (image_renderer.cuh:146-196): two overlapping fronto-parallel
    squares of different colours -- the nearer one's colour shows where they overlap, the farther one's elsewhere;
    a source pixel nearer than the render by more than the threshold (3-DoF) blacks the pixel out (depth 0, colour
    0); the depth equals orc_render_depth's."""
    W, H = 64, 48
    fx = fy = 50.0
    cx, cy = 32.0, 24.0
    proj = oracle.compute_proj(fx, fy, cx, cy, W, H)

    def square(z, half, dx):
        a = [[-half + dx, -half, z], [half + dx, -half, z], [half + dx, half, z]]
        b = [[-half + dx, -half, z], [half + dx, half, z], [-half + dx, half, z]]
        return np.array([a, b], np.float32).reshape(2, 9)

    tris = np.concatenate([square(1.0, 0.2, -0.1), square(0.8, 0.1, 0.1)])
    rgb = np.array([[200, 10, 10], [200, 10, 10], [10, 220, 30], [10, 220, 30]], np.uint8)
    pose = np.eye(4, dtype=np.float32) * 100.0
    pose[3, 3] = 1.0
    src = np.zeros((H, W), np.int32)
    src[0:10, 0:64] = 50  # a source surface at 50 cm over the top rows
    z, col = oracle.render_depth_color(tris, rgb, [4], pose.reshape(1, 16), np.zeros(1, np.int32), None, W, H, proj,
                                       src, None, 1.0)
    z0 = oracle.render_depth(tris, [4], pose.reshape(1, 16), np.zeros(1, np.int32), None, W, H, proj, src, None, 1.0)
    assert np.array_equal(z, z0)
    near = z[0] == 80
    far = z[0] == 100
    assert near.sum() > 50 and far.sum() > 50
    assert np.all(col[:, 0][:, near] == np.array([[10], [220], [30]]))
    assert np.all(col[:, 0][:, far] == np.array([[200], [10], [10]]))
    blocked = (src > 0) & (z[0] == 0)
    assert blocked.sum() > 0 and np.all(col[:, 0][:, blocked] == 0)
    assert np.all(col[:, 0][:, z[0] == 0] == 0)
