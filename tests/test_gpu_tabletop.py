"""GPU: the 3-DoF table-top search (f4) end to end -- bounded observed cloud, x / y / yaw grid with
IsValidPose, cylinder observed totals, cost_type 0 scoring and selection -- against the oracle on the
same candidate states."""
import math

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle
from perception_amd import synthetic as syn
from perception_amd.recognizer import CameraIntrinsics, ModelMetaData, preprocessing_transform
from perception_amd.tabletop import TableParams, TabletopRecognizer, pr2_gpu_params
from tests.helpers import oracle_render_fn

pytestmark = pytest.mark.gpu


def _scene(colors=None):
    names = ["003_cracker_box", "005_tomato_soup_can"]
    placements = [(0.60, -0.08, 0.4), (0.64, 0.10, 0.0)]
    bank = syn.model_bank(names)
    pre = [preprocessing_transform(m, six_dof=False) for m in bank.models]
    sc = syn.make_tabletop_scene(names, placements, pre, oracle_render_fn, table_height=0.7,
                                 rng=np.random.default_rng(4), colors=colors)
    return names, placements, sc


def test_tabletop_localization_matches_oracle():
    names, placements, sc = _scene()
    table = TableParams(x_min=0.48, x_max=0.76, y_min=-0.2, y_max=0.2, table_height=0.7, res=0.04)
    bank = {n: ModelMetaData(n, model=sc.bank.models[i]) for i, n in enumerate(names)}
    cam = CameraIntrinsics(sc.width, sc.height, sc.fx, sc.fy, sc.cx, sc.cy)
    rec = TabletopRecognizer(bank, cam, table, pr2_gpu_params(use_color_cost=False))
    res = rec.localize(names, sc.depth_raw, sc.camera_pose, sc.depth_factor)
    states = rec.generate_successor_states()
    assert len(states) > 100
    mats = rec._pose_in_cam(states)
    pm = np.array([s[0] for s in states], np.int32)
    tot = rec._obs_totals(states)
    obs = rec.obs_xyz_host
    # bounded observed cloud vs the oracle
    oxyz, _ = oracle.depth_to_cloud_bounded(sc.depth_raw, rec.params.gpu_stride, sc.cx, sc.cy, sc.fx, sc.fy,
                                            sc.depth_factor, rec.transform, rec.bounds)
    assert np.array_equal(obs, oxyz)
    src_cm = (sc.depth_raw.astype(np.float32) / (np.float32(sc.depth_factor) / np.float32(100))).astype(np.int32)
    rc, oc, df = oracle.evaluate(sc.bank.tris, sc.bank.tris_model_count, mats, pm, None, sc.width, sc.height, sc.proj,
                                 src_cm, None, rec.params.gpu_occlusion_threshold, rec.params.gpu_stride, sc.cx,
                                 sc.cy, sc.fx, sc.fy, 100.0, obs, None, None, tot, 0, True,
                                 rec.params.sensor_resolution)
    g_rc, g_oc, g_df = rec._last_costs
    assert np.array_equal(g_rc.view(np.uint32), rc.view(np.uint32))
    assert np.array_equal(g_oc.view(np.uint32), oc.view(np.uint32))
    bc, bi = oracle.select(rc, oc, pm, len(names))
    got = {m: (cost, idx) for m, cost, idx, _ in res}
    for m in range(len(names)):
        if bi[m] >= 0:
            assert got[m] == (int(bc[m]), int(bi[m]))
    # the box is found within one grid cell / yaw step of where it stands
    _, _, idx, cont = next(r for r in res if r[0] == 0)
    x, y, _, th = states[idx][2]
    assert abs(x - placements[0][0]) <= table.res and abs(y - placements[0][1]) <= table.res
    d = abs((th - placements[0][2] + math.pi) % (2 * math.pi) - math.pi)
    assert min(d, abs(d - math.pi)) <= table.theta_res  # a box is symmetric under a half turn
