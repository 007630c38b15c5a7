"""GPU: host orchestration (ObjectRecognizer / ComputeGreedyRenderPoses mirror) and the observed-side
preprocessing (f1) on the reference's own demo depth image, checked against the oracle."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle
from perception_amd import io, synthetic as syn
from perception_amd.core import PoseCore
from perception_amd.model import init_from_eigen_batch, matrix_to_quat_xyzw
from perception_amd.recognizer import (CameraIntrinsics, ModelMetaData, ObjectRecognizer, PerchParams,
                                       RecognitionInput)
from tests.helpers import oracle_render_fn

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_observed_cloud_on_reference_demo_depth():
    d = io.load_depth_png(os.path.join(G, "demo_depth.png"))
    cam = syn.CAM_640
    core = PoseCore(0)
    from perception_amd.model import compute_proj
    core.set_camera(640, 480, cam["fx"], cam["fy"], cam["cx"], cam["cy"],
                    compute_proj(cam["fx"], cam["fy"], cam["cx"], cam["cy"], 640, 480))
    mask = np.zeros_like(d, dtype=np.uint8)
    mask[100:300, 200:500] = 1
    mask[300:420, 100:250] = 2
    dev = torch.device("cuda", 0)
    for m in (None, mask):
        for stride in (8, 5, 1):
            xyz, lab = core.observed_cloud(torch.from_numpy(d).to(dev), None if m is None else torch.from_numpy(m).to(dev),
                                           stride, 10000.0)
            oxyz, _, olab = oracle.depth_to_cloud(d, stride, cam["cx"], cam["cy"], cam["fx"], cam["fy"], 10000.0,
                                                  label_mask=m)
            assert np.array_equal(xyz.cpu().numpy(), oxyz)
            assert np.array_equal(lab.cpu().numpy(), olab)


def _write_pose_lists(root, names, gts, rng, n=60):
    for k, name in enumerate(names):
        P = syn.candidate_poses(gts[k][:3, 3], n, rng, include=gts[k], num_viewpoints=20, inplane=4)
        rows = np.array([np.concatenate([T[:3, 3], matrix_to_quat_xyzw(T[:3, :3])]) for T in P])
        os.makedirs(os.path.join(root, name), exist_ok=True)
        io.write_poses_txt(os.path.join(root, name, "poses.txt"), rows, decimals=6)


@pytest.mark.parametrize("icp", [False, True])
def test_localize_objects_greedy_render_matches_oracle_pipeline(tmp_path, icp):
    names = ["003_cracker_box", "005_tomato_soup_can", "061_foam_brick"]
    rng = np.random.default_rng(5)
    gts = np.stack([syn.default_gt_pose(rng, c) for c in [(-0.12, 0.0, 0.8), (0.0, 0.05, 0.85), (0.13, -0.03, 0.75)]])
    sc = syn.make_scene(names, gts, oracle_render_fn, rng=rng)
    _write_pose_lists(str(tmp_path), names, gts, rng)
    bank = {n: ModelMetaData(n, model=sc.bank.models[i]) for i, n in enumerate(names)}
    cam = CameraIntrinsics(sc.width, sc.height, sc.fx, sc.fy, sc.cx, sc.cy)
    rec = ObjectRecognizer(bank, cam, PerchParams(icp_type=3 if icp else 0, gpu_batch_size=50))
    inp = RecognitionInput(names, sc.depth_raw, sc.mask, depth_factor=sc.depth_factor,
                           rendered_root_dir=str(tmp_path), use_icp=int(icp))
    res = rec.localize_objects_greedy_render(inp)
    assert res.model_names == names
    # oracle pipeline on the same candidate states
    states = rec.generate_successor_states(inp)
    mats = rec._pose_in_cam(states)
    pm = np.array([s[0] for s in states], np.int32)
    pl = np.array([s[1] for s in states], np.int32)
    xyz, lab = rec.obs_xyz_host, rec.obs_label_host
    order = np.argsort(lab, kind="stable")
    oxyz, olab = xyz[order], lab[order]
    ls = np.array([np.searchsorted(olab, L, "left") for L in range(3)], np.int32)
    le = np.array([np.searchsorted(olab, L, "right") for L in range(3)], np.int32)
    tot = rec.segmented_count[pl]
    src = sc.src_depth_cm
    if icp:
        ocov = np.zeros((len(oxyz), 6))
        for L in range(3):
            ocov[ls[L]:le[L]] = oracle.covariances(oxyz[ls[L]:le[L]])
        adj, _, rc, oc, df = oracle.evaluate_icp(sc.bank.tris, sc.bank.tris_model_count, mats, pm, pl, sc.width,
                                                 sc.height, sc.proj, src, sc.mask, 1.0, 8, sc.cx, sc.cy, sc.fx, sc.fy,
                                                 100.0, oxyz, ocov, ls, le, tot, 2, True, 0.01)
    else:
        rc, oc, df = oracle.evaluate(sc.bank.tris, sc.bank.tris_model_count, mats, pm, pl, sc.width, sc.height,
                                     sc.proj, src, sc.mask, 1.0, 8, sc.cx, sc.cy, sc.fx, sc.fy, 100.0, oxyz, ls, le,
                                     tot, 2, True, 0.01)
        adj = mats
    bc, bi = oracle.select(rc, oc, pm, 3)
    assert res.indices == [int(i) for i in bi if i >= 0]
    assert res.costs == [int(c) for c, i in zip(bc, bi) if i >= 0]
    for k, i in enumerate(res.indices):
        T = np.asarray(adj[i], np.float32).reshape(4, 4)
        assert np.allclose(res.detected_poses[k][:3], T[:3, 3] / 100.0, atol=1e-6)
    # every object is found near its GT pose
    for k in range(len(res.model_names)):
        assert np.linalg.norm(res.detected_poses[k][:3] - gts[k][:3, 3]) < 0.05
    rec.write_outputs(res, str(tmp_path / "out"))
    back = io.read_output_poses(str(tmp_path / "out" / "output_poses.txt"))
    assert [b.name for b in back] == names
    # ADD-S AUC (north star: within 0.1 of the reference): the GPU pipeline's selected poses, scored with the
    # GPU ADD-S kernel, against the oracle pipeline's selected poses scored with the f64 CPU ADD-S
    from perception_amd import metrics
    from perception_amd.model import to_eigen
    g_err, o_err = [], []
    for k, i in enumerate(bi):
        pts = np.unique(sc.bank.models[k].tris.reshape(-1, 3), axis=0)
        est_gpu = np.asarray(res.object_transforms[k], np.float64)
        est_orc = to_eigen(np.asarray(adj[i], np.float32)).astype(np.float64)
        _, s_gpu = metrics.pose_distances(rec.core, pts, gts[k][None], est_gpu[None])
        _, s_orc = oracle.pose_distances(pts, gts[k][None], est_orc[None])
        g_err.append(float(s_gpu[0].item()))
        o_err.append(float(s_orc[0]))
    auc_gpu = metrics.compute_pose_metrics(np.array(g_err))["auc"]
    auc_orc = metrics.compute_pose_metrics(np.array(o_err))["auc"]
    assert abs(auc_gpu - auc_orc) <= 0.1, (auc_gpu, auc_orc)


def test_device_state_path_equals_host_state_path():
    """the 6-DoF search builds its per-state inputs on the device (_successor_states_device,
    _state_poses_dev, _pose_labels_dev, _obs_totals_dev); they equal the host path's (generate_successor_states,
    _pose_in_cam / _poses_device, _pose_labels, _obs_totals) element for element -- including a model that is not
    among the segmented objects (required object id = len(segmented), observed total 0), kept here by a zero
    neighbour threshold."""
    names = ["003_cracker_box", "005_tomato_soup_can", "061_foam_brick"]
    extra = "024_bowl"
    rng = np.random.default_rng(21)
    gts = np.stack([syn.default_gt_pose(rng, c) for c in [(-0.12, 0.0, 0.8), (0.0, 0.05, 0.85), (0.13, -0.03, 0.75)]])
    sc = syn.make_scene(names, gts, oracle_render_fn, rng=rng)
    bank = {n: ModelMetaData(n, model=sc.bank.models[i]) for i, n in enumerate(names)}
    bank[extra] = ModelMetaData(extra, model=syn.ycb_proxy(extra))
    cam = CameraIntrinsics(sc.width, sc.height, sc.fx, sc.fy, sc.cx, sc.cy)
    rec = ObjectRecognizer(bank, cam, PerchParams(icp_type=0, min_neighbor_points_for_valid_pose=0))
    rec.set_static_input(names + [extra])
    lists = {}
    for k, name in enumerate(names + [extra]):
        P = syn.candidate_poses(gts[min(k, 2)][:3, 3], 40, rng, num_viewpoints=10, inplane=4)
        lists[name] = np.array([np.concatenate([T[:3, 3], matrix_to_quat_xyzw(T[:3, :3])]) for T in P])
    inp = RecognitionInput(names, sc.depth_raw, sc.mask, depth_factor=sc.depth_factor, pose_lists=lists)
    rec.set_input(inp)  # segmented objects: the three scene names; the bowl has no label
    model_d, req_d, pose_d = rec._successor_states_device(inp)
    host = rec.generate_successor_states(inp)
    assert np.array_equal(model_d.cpu().numpy(), host.model) and np.array_equal(req_d.cpu().numpy(), host.req)
    assert np.array_equal(pose_d.cpu().numpy(), host.pose)
    assert (host.model == 3).sum() == 40 and (host.req[host.model == 3] == 3).all()  # the unsegmented model's states
    poses_dev = rec._state_poses_dev(pose_d, model_d).cpu().numpy()
    assert np.array_equal(poses_dev.view(np.uint32), rec._poses_device(host).cpu().numpy().view(np.uint32))
    assert np.array_equal(poses_dev.view(np.uint32), rec._pose_in_cam(host).view(np.uint32))
    assert np.array_equal(rec._pose_labels_dev(req_d).cpu().numpy(), rec._pose_labels(host).cpu().numpy())
    tot_dev, tot_host = rec._obs_totals_dev(req_d).cpu().numpy(), rec._obs_totals(host)
    assert np.array_equal(tot_dev.view(np.uint32), tot_host.view(np.uint32))
    assert (tot_host[host.model == 3] == 0).all()
