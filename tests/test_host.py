"""Host-side logic: mat4x4 helpers, key encoding, sharding, synthetic proxies."""
import numpy as np

from perception_amd import synthetic as syn
from perception_amd.core import decode_keys, encode_key
from perception_amd.distributed import shard_range
from perception_amd.model import (init_from_eigen, init_from_eigen_batch, matrix_to_quat_xyzw, pose_matrix,
                                  quat_xyzw_to_matrix, to_eigen)


def test_mat4x4_scaling_roundtrip():
    T = pose_matrix([0.1, -0.2, 0.8], [0.1, 0.2, 0.3, 0.9])
    m = init_from_eigen(T, 100)
    assert m.dtype == np.float32 and m.shape == (16,)
    assert np.allclose(m[:12].reshape(3, 4), T[:3] * 100, rtol=1e-6)
    assert np.array_equal(m[12:], np.array([0, 0, 0, 1], np.float32))
    assert np.allclose(to_eigen(m, 100), T, atol=1e-6)
    assert np.array_equal(init_from_eigen_batch(np.stack([T, T]))[1], m)


def test_quaternion_roundtrip():
    rng = np.random.default_rng(0)
    for _ in range(20):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        R = quat_xyzw_to_matrix(q)
        assert np.allclose(R @ R.T, np.eye(3), atol=1e-12)
        q2 = matrix_to_quat_xyzw(R)
        assert np.allclose(np.abs(np.dot(q, q2)), 1.0, atol=1e-9)


def test_key_encoding_orders_like_the_reference_scan():
    keys = [encode_key(c, i) for c, i in [(7, 5), (7, 3), (6, 100), (0, 2**31 - 2), (-5, 1)]]
    order = np.argsort(keys)
    assert list(order) == [4, 3, 2, 1, 0]
    cost, idx = decode_keys(np.array(keys, np.int64))
    assert list(cost) == [7, 7, 6, 0, -5] and list(idx) == [5, 3, 100, 2**31 - 2, 1]
    none_cost, none_idx = decode_keys(np.array([0x7FFFFFFFFFFFFFFF], np.int64))
    assert none_cost[0] == 2**31 - 1 and none_idx[0] == -1
    assert all(0 <= k < 2**63 - 1 for k in keys)


def test_shard_range_covers_exactly():
    for total in (0, 1, 7, 10000, 200003):
        for world in (1, 2, 3, 8):
            parts = [shard_range(total, r, world) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == total
            assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1


def test_cracker_box_proxy_has_12288_triangles():
    m = syn.ycb_proxy("003_cracker_box")
    assert m.tris.shape == (12288, 9)
    ext = m.tris.reshape(-1, 3).max(0) - m.tris.reshape(-1, 3).min(0)
    assert np.allclose(ext, [0.060, 0.158, 0.210], atol=1e-6)
    assert (m.colors == 128).all()


def test_all_21_proxies_build():
    bank = syn.model_bank(list(syn.YCB_PROXIES))
    assert len(bank.models) == 21
    assert bank.tris.shape[0] == bank.tris_model_count.sum()


def test_c4_scene_every_object_visible():
    """C4's 21-object scene (workloads.object_centers, the GT rotation of workloads.build), rendered by the
    oracle: every object keeps most of its unoccluded stride-8 samples, so every model has a findable pose."""
    import oracle
    from perception_amd import workloads

    def rf(tris, cnt, p16, pm, W, H, proj):
        return oracle.render_depth(tris, cnt, p16, pm, None, W, H, proj, np.zeros((H, W), np.int32), None)

    names = list(syn.YCB_PROXIES)
    rng = np.random.default_rng(syn.SEED)
    gts = np.stack([syn.default_gt_pose(rng, c) for c in workloads.object_centers(len(names))])
    sc = syn.make_scene(names, gts, rf, rng=rng)
    alone = rf(sc.bank.tris, sc.bank.tris_model_count, init_from_eigen_batch(gts), np.arange(len(names), dtype=np.int32),
               sc.width, sc.height, sc.proj)
    for k in range(len(names)):
        vis = int((sc.mask[::8, ::8] == k + 1).sum())
        tot = int((alone[k][::8, ::8] > 0).sum())
        assert vis >= 5 and vis >= 0.9 * tot, (names[k], vis, tot)


def test_candidate_poses_include_gt_and_are_rigid():
    rng = np.random.default_rng(1)
    gt = syn.default_gt_pose(rng)
    P = syn.candidate_poses(gt[:3, 3], 1000, rng, include=gt)
    assert P.shape == (1000, 4, 4)
    assert np.array_equal(P[1000 // 3], gt)
    R = P[:, :3, :3]
    assert np.allclose(np.einsum("nij,nkj->nik", R, R), np.eye(3), atol=1e-9)


def test_batched_pose_building_matches_per_state():
    """The recognizers' vectorised pose building: rotations bit-equal to the per-state quaternion
    conversion, the 4x4 chain bit-equal to the index-order product loop and within 1e-12 of numpy's BLAS
    matmul; the 3-DoF builder equal to yaw_pose_matrix state by state."""
    import numpy as np
    from perception_amd.model import chain_matmul_batch, pose_matrix, pose_matrix_batch
    from perception_amd.tabletop import yaw_pose_matrix

    rng = np.random.default_rng(3)
    n = 300
    P = np.concatenate([rng.normal(size=(n, 3)), rng.normal(size=(n, 4))], 1)
    A = rng.normal(size=(4, 4))
    B = rng.normal(size=(n, 4, 4))
    T = pose_matrix_batch(P[:, :3], P[:, 3:])
    assert np.array_equal(T, np.stack([pose_matrix(p[:3], p[3:]) for p in P]))

    def mm(X, Y):
        Z = np.empty((4, 4))
        for r in range(4):
            for c in range(4):
                Z[r, c] = ((X[r, 0] * Y[0, c] + X[r, 1] * Y[1, c]) + X[r, 2] * Y[2, c]) + X[r, 3] * Y[3, c]
        return Z

    out = chain_matmul_batch(A, T, B)
    for i in range(0, n, 37):
        assert np.array_equal(out[i], mm(A, mm(T[i], B[i])))  # search_env.cpp:1567-1571 grouping
    assert np.allclose(out, np.stack([A @ T[i] @ B[i] for i in range(n)]), rtol=0, atol=1e-12)
    # the quaternion norm in Eigen's packet order (x^2 + z^2) + (y^2 + w^2)
    x, y, z, w = P[:, 3], P[:, 4], P[:, 5], P[:, 6]
    nrm = np.sqrt((x * x + z * z) + (y * y + w * w))
    assert np.array_equal(T[:, 2, 2], 1 - 2 * ((x / nrm) * (x / nrm) + (y / nrm) * (y / nrm)))
    # 3-DoF: the yaw quaternion path
    xyz = rng.uniform(-1, 1, (n, 3))
    yaw = rng.uniform(-7, 7, n)
    from perception_amd.tabletop import normalize_angle_positive
    import math
    q = np.array([(0.0, 0.0, math.sin(normalize_angle_positive(y) / 2.0), math.cos(normalize_angle_positive(y) / 2.0))
                  for y in yaw])
    assert np.array_equal(pose_matrix_batch(xyz, q), np.stack([yaw_pose_matrix(*xyz[i], yaw[i]) for i in range(n)]))


def test_quaternion_from_matrix_is_eigens_algorithm():
    """quat_from_matrix_eigen_batch (Eigen::Quaternion(Matrix3), both branches, float and double) against scipy's
    rotation-to-quaternion up to sign and rounding, and branch by branch against a scalar transcription."""
    from scipy.spatial.transform import Rotation

    from perception_amd.model import quat_from_matrix_eigen_batch

    rng = np.random.default_rng(3)
    R = Rotation.random(4000, random_state=4).as_matrix()
    R[:4] = [np.eye(3), np.diag([1.0, -1.0, -1.0]), np.diag([-1.0, 1.0, -1.0]), np.diag([-1.0, -1.0, 1.0])]
    for dt, tol in ((np.float64, 1e-12), (np.float32, 3e-7)):
        q = quat_from_matrix_eigen_batch(R, dt)
        assert q.dtype == dt
        ref = Rotation.from_matrix(R).as_quat()  # x y z w
        sgn = np.sign(np.sum(q * ref, 1))[:, None]
        assert np.abs(q - sgn * ref).max() < tol * 10
    # the non-positive-trace branch picks the first largest diagonal entry (Eigen's i, j, k)
    m = np.array([[-0.5, 0.0, 0.0], [0.0, -0.5, 0.0], [0.0, 0.0, 0.0]])
    tr = m.trace()
    assert tr <= 0
    q = quat_from_matrix_eigen_batch(m[None], np.float64)[0]
    t = np.sqrt(((m[2, 2] - m[0, 0]) - m[1, 1]) + 1.0)
    assert q[2] == 0.5 * t and q[3] == (m[1, 0] - m[0, 1]) * (0.5 / t)


def test_so3_log_matches_rotation_vectors():
    from scipy.spatial.transform import Rotation

    from perception_amd.model import so3_log_batch

    q = Rotation.random(2000, random_state=8).as_quat()
    q = q * np.where(q[:, 3:] < 0, -1.0, 1.0)  # w >= 0: the rotation vector of angle <= pi
    q[0] = [0.0, 0.0, 0.0, 1.0]          # identity: the small-angle branch
    q[1] = [1e-7, 0.0, 0.0, 1.0]
    q[2] = [0.0, 1.0, 0.0, 1e-7]         # ~pi about y: |w| < eps, +pi / n
    want = Rotation.from_quat(q).as_rotvec()
    got = so3_log_batch(q.astype(np.float32), np.float32).astype(np.float64)
    assert np.abs(got - want).max() < 2e-5
    assert np.abs(got[2] - [0.0, np.pi, 0.0]).max() < 1e-6
    # w = 0 exactly takes -pi / n (Sophus: w > 0 is false)
    assert np.abs(so3_log_batch(np.array([[0.0, 1.0, 0.0, 0.0]]))[0] - [0.0, -np.pi, 0.0]).max() < 1e-6


def test_cvtt_i32_is_x86_truncation():
    from perception_amd.recognizer import cvtt_i32

    x = np.array([1.9, -1.9, -0.5, 0.0, 99.99, np.nan, np.inf, -np.inf, 3e9, -3e9, -1.0], np.float32)
    assert cvtt_i32(x).tolist() == [1, -1, 0, 0, 99, -2**31, -2**31, -2**31, -2**31, -2**31, -1]


def test_cost_dump_format(tmp_path):
    """cost_dump.json as nlohmann::json prints it with setw(4): sorted keys, four-space indent, trailing newline."""
    from perception_amd import io as pio

    p = tmp_path / "cost_dump.json"
    entry = {"id": 3, "target_cost": 4, "source_cost": 7, "total_cost": 11, "transform": [1.0] * 16,
             "translation": [0.1, 0.2, 0.8], "quaternion": [0.0, 0.0, 0.0, 1.0], "lie_rotation": [0.0, 0.0, 0.0]}
    pio.write_cost_dump(str(p), [entry])
    text = p.read_text()
    assert text.startswith('{\n    "poses": [\n        {\n            "id": 3,\n            "lie_rotation": [\n')
    assert text.endswith("}\n")
    assert pio.read_cost_dump(str(p)) == [entry]
    pio.write_cost_dump(str(p), [])
    assert p.read_text() == '{\n    "poses": []\n}\n'
