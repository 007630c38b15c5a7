"""IsValidPose (search_env.cpp:309-410) on the CPU: the search radius and PCL's radius-search count.

The reference counts neighbours with pcl::search::KdTree (FLANN KDTreeSingleIndex, exact): float PointXYZ query
and points, radius passed squared as float(r * r), L2_Simple's float sum ((0 + dx^2) + dy^2) + dz^2 and a strict
dist < r^2.  The restatement here is plain numpy float32 with an explicit loop over the points; the product path
(perception_amd.recognizer.radius_counts) runs torch elementwise ops on the recognizer's device.
"""
import math

import numpy as np
import pytest

from perception_amd.recognizer import (ModelMetaData, ObjectRecognizer, PerchParams, radius_counts,
                                       valid_pose_mask)
from perception_amd import synthetic as syn
from tests.helpers import SceneCase


def _pcl_counts(queries, points, radius):
    q = np.asarray(queries, np.float64).astype(np.float32)
    p = np.asarray(points, np.float32)
    r2 = np.float32(radius * radius)
    out = []
    for qi in q:
        d = np.zeros(len(p), np.float32)
        for a in range(3):
            diff = np.float32(qi[a]) - p[:, a]
            d = d + diff * diff
        out.append(int((d < r2).sum()))
    return np.array(out)


@pytest.fixture(scope="module")
def segment():
    case = SceneCase(("003_cracker_box", "005_tomato_soup_can"), n_poses=4, seed=4)
    return case.obs_xyz[case.label_start[0]:case.label_end[0]], case


def test_radius_counts_match_pcl_float_semantics(segment):
    seg, _ = segment
    rng = np.random.default_rng(3)
    c = seg.mean(0).astype(np.float64)
    queries = c + rng.normal(scale=0.05, size=(200, 3))
    for r in (0.02, 0.0566, 0.11, 0.3):
        assert np.array_equal(radius_counts(queries, seg, r, "cpu"), _pcl_counts(queries, seg, r))


def test_radius_boundary_is_strict_in_float():
    """A point at exactly float distance r^2 is not a neighbour; one float ulp inside is."""
    r = 0.05
    r2 = np.float32(r * r)
    q = np.array([[0.1, 0.2, 0.7]])
    qf = q.astype(np.float32)[0]
    # walk a point along x until its float squared distance crosses r2
    x = np.float32(qf[0] + np.float32(r))
    pts = []
    for _ in range(40):
        d = (np.float32(qf[0]) - x) * (np.float32(qf[0]) - x)
        pts.append((x, d))
        x = np.nextafter(x, np.float32(0.0))
    on = [p for p, d in pts if d == r2]
    inside = [p for p, d in pts if d < r2]
    assert inside
    cand = np.array([[inside[0], qf[1], qf[2]]] + ([[on[0], qf[1], qf[2]]] if on else []), np.float32)
    got = radius_counts(q, cand, r, "cpu")[0]
    assert got == 1 == _pcl_counts(q, cand, r)[0]


def _recognizer_stub(res=0.04, model_specific=False, model_res=0.04, name="003_cracker_box"):
    rec = ObjectRecognizer.__new__(ObjectRecognizer)
    m = syn.ycb_proxy(name)
    rec.bank = {name: ModelMetaData(name, model=m, search_resolution=model_res)}
    rec.params = PerchParams(search_resolution=res, use_model_specific_search_resolution=model_specific)
    rec.models = [m]
    rec.model_names = [name]
    rec.device = "cpu"
    return rec


def test_search_radius_is_max_of_inflated_radius_and_cell_radius():
    """search_rad = max(inflation * circumscribed radius 3D, hypot(res / 2, res / 2)) (search_env.cpp:343-390)."""
    rec = _recognizer_stub(res=0.04)
    dims = rec.models[0].tris.reshape(-1, 3).max(0).astype(np.float64) - rec.models[0].tris.reshape(-1, 3).min(0)
    circ = max(dims) / 2.0
    infl = 1.0 + 0.01 / (min(dims[0], dims[1]) / 2.0)
    assert rec._search_radius(0) == max(infl * circ, math.hypot(0.02, 0.02))
    assert rec._search_radius(0) == infl * circ  # a 21 cm box: the object term
    coarse = _recognizer_stub(res=0.5)
    assert coarse._search_radius(0) == math.hypot(0.25, 0.25)  # a coarse grid: the cell term
    own = _recognizer_stub(res=0.5, model_specific=True, model_res=0.04)
    assert own._search_radius(0) == rec._search_radius(0)


def test_valid_pose_mask_against_restatement(segment):
    seg, _ = segment
    rng = np.random.default_rng(8)
    c = seg.mean(0).astype(np.float64)
    t = c + rng.normal(scale=0.06, size=(300, 3))
    for need in (1, 30, 60):
        for r in (0.03, 0.08):
            got = valid_pose_mask(t, seg, r, need, "cpu")
            want = _pcl_counts(t, seg, r) >= need if len(seg) >= need else np.zeros(len(t), bool)
            assert np.array_equal(got, want)
    assert not valid_pose_mask(t[:3], seg[:5], 1.0, 30, "cpu").any()  # fewer points than needed
