"""3-DoF table-top host logic (f4): ContPose yaw transform, the x / y / yaw grid and its validity filter."""
import math

import numpy as np
from scipy.spatial.transform import Rotation

from perception_amd.tabletop import (TableParams, circumscribed_radius, grid_states, normalize_angle_positive,
                                     yaw_pose_matrix)


def test_normalize_angle_positive():
    assert normalize_angle_positive(0.0) == 0.0
    assert abs(normalize_angle_positive(-0.5) - (2 * math.pi - 0.5)) < 1e-15
    assert abs(normalize_angle_positive(7.0) - (7.0 - 2 * math.pi)) < 1e-15
    assert 0.0 <= normalize_angle_positive(2 * math.pi) < 2 * math.pi


def test_yaw_pose_matrix_is_translation_times_rz():
    for yaw in (0.0, 0.3926991, 1.0, 3.5, 6.0):
        T = yaw_pose_matrix(0.5, -0.2, 0.7, yaw)
        assert np.allclose(T[:3, :3], Rotation.from_euler("z", yaw).as_matrix(), atol=1e-15)
        assert np.array_equal(T[:3, 3], [0.5, -0.2, 0.7])


def test_grid_states_loop_semantics_and_validity():
    tb = TableParams(x_min=0.5, x_max=0.62, y_min=-0.04, y_max=0.04, table_height=0.7, res=0.04, theta_res=0.3926991)
    # repeated double addition: 0.5, 0.54, 0.58, 0.62000000000000011 (> 0.62 -> not visited)
    xs = sorted({round(s[2][0], 12) for s in grid_states(tb, 0, [0.1, 0.1, 0.2], np.zeros((0, 2)), 0)})
    assert xs == [0.5, 0.54, 0.58]
    thetas = [s[2][3] for s in grid_states(tb, 0, [0.1, 0.1, 0.2], np.zeros((0, 2)), 0)][:17]
    assert len({round(t, 9) for t in thetas}) == 16  # 0 .. 15 * theta_res < 2 pi
    # validity: 30 projected points around (0.54, 0.0) only
    rng = np.random.default_rng(0)
    pts = np.array([0.54, 0.0]) + rng.uniform(-0.01, 0.01, (30, 2))
    st = grid_states(tb, 3, [0.06, 0.06, 0.2], pts, 30)
    centres = {(round(s[2][0], 6), round(s[2][1], 6)) for s in st}
    rad = max(circumscribed_radius([0.06, 0.06]), math.hypot(0.02, 0.02))
    for cx, cy in centres:
        assert (np.hypot(pts[:, 0] - cx, pts[:, 1] - cy) <= rad).sum() >= 30
    assert (0.54, 0.0) in centres and all(s[0] == 3 and s[1] == -1 for s in st)
    # semi-symmetric: yaw stops after the first yaw above pi + theta_res
    half = grid_states(tb, 0, [0.06, 0.06, 0.2], pts, 30, symmetry_mode=1)
    per_cell = len(half) // len(centres)
    assert per_cell == sum(1 for k in range(16) if k * 0.3926991 <= math.pi + 0.3926991)


def test_median_blur_u8_matches_replicate_border_median():
    """cv::medianBlur semantics for 8-bit depth (search_env.cpp:5922): the window median with the border
    replicated -- scipy's median_filter(mode='nearest') is the same definition."""
    from scipy.ndimage import median_filter

    from perception_amd.tabletop import median_blur_u8

    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, size=(61, 83), dtype=np.uint8)
    img[10:30, 20:50] = 0  # depth holes
    for k in (1, 3, 5, 17):
        got = median_blur_u8(img, k)
        want = img if k == 1 else median_filter(img, size=k, mode="nearest")
        assert np.array_equal(got, want), k
