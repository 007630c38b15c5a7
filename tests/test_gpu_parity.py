"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle on the same inputs.

Bar: bit-exact for every integer / index output (z-buffers, clouds' order, argmin) and for the float
costs (same explicit operation order on both sides, no FMA contraction).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle
from perception_amd import synthetic as syn
from perception_amd.core import PoseCore, decode_keys
from perception_amd.model import init_from_eigen_batch
from tests.helpers import SceneCase

pytestmark = pytest.mark.gpu


def _bits_equal(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape:
        return False
    if a.dtype.kind == "f":
        return np.array_equal(a.view(np.uint32), b.view(np.uint32)) or np.array_equal(a, b, equal_nan=True)
    return np.array_equal(a, b)


def _setup(case: SceneCase, stride=8):
    sc = case.scene
    core = PoseCore(0)
    core.upload_meshes(sc.bank.tris, sc.bank.tris_model_count)
    core.set_camera(sc.width, sc.height, sc.fx, sc.fy, sc.cx, sc.cy, sc.proj)
    dev = torch.device("cuda", 0)
    t = {
        "raw": torch.from_numpy(sc.depth_raw).to(dev),
        "mask": torch.from_numpy(sc.mask).to(dev),
        "src": torch.from_numpy(sc.src_depth_cm).to(dev),
        "poses": torch.from_numpy(case.poses).to(dev),
        "pm": torch.from_numpy(case.pose_model).to(dev),
        "pl": torch.from_numpy(case.pose_label).to(dev),
        "tot": torch.from_numpy(case.pose_obs_total).to(dev),
    }
    xyz, lab = core.observed_cloud(t["raw"], t["mask"], stride, sc.depth_factor)
    t["obs_xyz"], t["obs_lab"] = xyz, lab
    core.set_observation(t["src"], t["mask"], xyz, lab, 0.01)
    return core, t


@pytest.fixture(scope="module")
def one_object():
    case = SceneCase(("003_cracker_box",), n_poses=96)
    core, t = _setup(case)
    return case, core, t


@pytest.fixture(scope="module")
def three_objects():
    case = SceneCase(("003_cracker_box", "005_tomato_soup_can", "061_foam_brick"), n_poses=48)
    core, t = _setup(case)
    return case, core, t


def test_observed_cloud_matches_oracle(one_object):
    case, core, t = one_object
    xyz, lab = t["obs_xyz"].cpu().numpy(), t["obs_lab"].cpu().numpy()
    assert _bits_equal(xyz, case.obs_xyz_raw)
    assert _bits_equal(lab, case.obs_label_raw)


@pytest.mark.parametrize("fixture", ["one_object", "three_objects"])
def test_render_full_zbuffer_bit_exact(fixture, request):
    case, core, t = request.getfixturevalue(fixture)
    sc = case.scene
    n = min(24, len(case.poses))
    zb = core.render(t["poses"][:n], t["pm"][:n], t["pl"][:n]).cpu().numpy()
    ref = oracle.render_depth(sc.bank.tris, sc.bank.tris_model_count, case.poses[:n], case.pose_model[:n],
                              case.pose_label[:n], sc.width, sc.height, sc.proj, sc.src_depth_cm, sc.mask, 1.0)
    assert (ref > 0).sum() > 0
    mism = np.argwhere(zb != ref)
    assert len(mism) == 0, f"{len(mism)} mismatching pixels, first {mism[:5]}"


def test_render_3dof_occlusion_threshold(one_object):
    case, core, t = one_object
    sc = case.scene
    n = 16
    zb = core.render(t["poses"][:n], t["pm"][:n], None, occlusion_threshold=1.0).cpu().numpy()
    ref = oracle.render_depth(sc.bank.tris, sc.bank.tris_model_count, case.poses[:n], case.pose_model[:n], None,
                              sc.width, sc.height, sc.proj, sc.src_depth_cm, None, 1.0)
    assert np.array_equal(zb, ref)


@pytest.mark.parametrize("fixture", ["one_object", "three_objects"])
def test_evaluate_costs_bit_exact(fixture, request):
    case, core, t = request.getfixturevalue(fixture)
    rc, oc, df = core.evaluate(t["poses"], t["pm"], t["pl"], t["tot"], cost_type=2, stride=case.stride)
    torch.cuda.synchronize()
    orc, ooc, odf = case.oracle_costs(cost_type=2)
    rc, oc, df = rc.cpu().numpy(), oc.cpu().numpy(), df.cpu().numpy()
    bad = np.nonzero(~((rc == orc) & (oc == ooc) & (df == odf)))[0]
    assert len(bad) == 0, f"{len(bad)} poses differ, e.g. {bad[:5]}: gpu {rc[bad[:3]]} {oc[bad[:3]]} oracle {orc[bad[:3]]} {ooc[bad[:3]]}"
    # the GT pose (written at n//3 of each object's block) must be a perfect fit
    assert (rc >= 0).sum() > len(rc) // 4


def test_evaluate_3dof_bit_exact(one_object):
    case, core, t = one_object
    tot = torch.full((len(case.poses),), float(len(case.obs_xyz)), device=t["poses"].device)
    rc, oc, df = core.evaluate(t["poses"], t["pm"], None, tot, cost_type=0, stride=case.stride)
    orc, ooc, odf = case.oracle_costs(cost_type=0)
    assert _bits_equal(rc.cpu().numpy(), orc)
    assert _bits_equal(oc.cpu().numpy(), ooc)
    assert _bits_equal(df.cpu().numpy(), odf)


def test_sampled_zbuffer_equals_full_render(one_object):
    case, core, t = one_object
    sc = case.scene
    n = 24
    s = case.stride
    hs, ws = (sc.height + s - 1) // s, sc.width // s
    dbg = torch.empty((n, hs, ws), dtype=torch.int32, device=t["poses"].device)
    core.evaluate(t["poses"][:n], t["pm"][:n], t["pl"][:n], t["tot"][:n], cost_type=2, stride=s, dbg_zs=dbg)
    full = core.render(t["poses"][:n], t["pm"][:n], t["pl"][:n]).cpu().numpy()
    assert np.array_equal(dbg.cpu().numpy(), full[:, ::s, ::s])


def test_depth_to_cloud_matches_oracle(one_object):
    case, core, t = one_object
    sc = case.scene
    n = 12
    zb = core.render(t["poses"][:n], t["pm"][:n], t["pl"][:n])
    xyz, pose, lab = core.depth_to_cloud(zb, case.stride, 100.0, pose_label=t["pl"][:n])
    oxyz, opose, olab = oracle.depth_to_cloud(zb.cpu().numpy(), case.stride, sc.cx, sc.cy, sc.fx, sc.fy, 100.0,
                                              pose_label=case.pose_label[:n])
    assert _bits_equal(xyz.cpu().numpy(), oxyz)
    assert np.array_equal(pose.cpu().numpy(), opose)
    assert np.array_equal(lab.cpu().numpy(), olab)


def test_depth_to_cloud_colours_and_dc_index(one_object):
    """Stage CLOUD's debug outputs (renderer.cu:1821-1847, pcore_depth_to_cloud_ex): result_dc_index is the reference's
    exclusive scan of the stride mask over every pixel of the N z-buffers (compute_point_clouds.cuh:267-292), and
    result_cloud_color gathers the colour planes at the points (:163-165); the points themselves are the plain call's.
    Restated here in numpy on random colour planes, with and without a label mask."""
    case, core, t = one_object
    sc = case.scene
    s = case.stride
    n = 9
    zb = core.render(t["poses"][:n], t["pm"][:n], t["pl"][:n])
    rng = np.random.default_rng(3)
    planes = rng.integers(0, 256, size=(3, n, sc.height, sc.width), dtype=np.uint8)
    dev = zb.device
    for label_mask in (None, t["mask"]):
        m = n if label_mask is None else 1
        z = zb[:m]
        pl = t["pl"][:m]
        xyz, pose, lab, col, dc = core.depth_to_cloud(z, s, 100.0, label_mask=label_mask, pose_label=pl,
                                                      color_planes=torch.from_numpy(planes[:, :m].copy()).to(dev),
                                                      dc_index=True)
        pxyz, ppose, plab = core.depth_to_cloud(z, s, 100.0, label_mask=label_mask, pose_label=pl)
        assert _bits_equal(xyz.cpu().numpy(), pxyz.cpu().numpy())
        assert np.array_equal(pose.cpu().numpy(), ppose.cpu().numpy())
        assert np.array_equal(lab.cpu().numpy(), plab.cpu().numpy())
        zn = z.cpu().numpy()
        mask = np.zeros(zn.shape, bool)
        mask[:, ::s, ::s] = zn[:, ::s, ::s] > 0
        if label_mask is not None:
            mask &= label_mask.cpu().numpy()[None] > 0
        flat = mask.ravel().astype(np.int64)
        want_dc = (np.cumsum(flat) - flat).reshape(zn.shape)
        assert np.array_equal(dc.cpu().numpy(), want_dc)
        assert len(xyz) == flat.sum() > 0
        want_col = planes[:, :m].reshape(3, -1)[:, mask.ravel()]
        assert np.array_equal(col.cpu().numpy(), want_col)


def test_select_matches_oracle(three_objects):
    case, core, t = three_objects
    rc, oc, df = core.evaluate(t["poses"], t["pm"], t["pl"], t["tot"], cost_type=2, stride=case.stride)
    keys = core.select(rc, oc, t["pm"], case.K, index_base=1000)
    cost, idx = decode_keys(keys)
    ocost, oidx = oracle.select(rc.cpu().numpy(), oc.cpu().numpy(), case.pose_model, case.K, 1000)
    assert np.array_equal(cost, ocost)
    assert np.array_equal(idx, oidx)


def test_select_ties_lowest_index():
    core = PoseCore(0)
    dev = torch.device("cuda", 0)
    rc = torch.tensor([5.0, 3.0, 3.0, -1.0, 3.0, 90.0], device=dev)
    oc = torch.tensor([5.0, 4.0, 4.0, 0.0, 4.0, 10.0], device=dev)
    pm = torch.tensor([0, 0, 0, 0, 1, 1], dtype=torch.int32, device=dev)
    cost, idx = decode_keys(core.select(rc, oc, pm, 2))
    ocost, oidx = oracle.select(rc.cpu().numpy(), oc.cpu().numpy(), pm.cpu().numpy(), 2)
    assert list(cost) == [7, 7] and list(idx) == [1, 4]
    assert np.array_equal(cost, ocost) and np.array_equal(idx, oidx)


def test_edge_poses(one_object):
    """Poses behind the camera, straddling z = 0, out of view and very close (large triangles)."""
    case, core, t = one_object
    sc = case.scene
    P = []
    for tz in (-0.5, 0.0, 0.02, 0.12, 0.25, 3.0):
        T = np.eye(4)
        T[:3, 3] = (0.0, 0.0, tz)
        P.append(T)
    T = np.eye(4); T[:3, 3] = (2.0, 0.0, 0.8); P.append(T)       # out of view
    T = np.eye(4); T[:3, 3] = (0.0, 0.0, 0.10); T[:3, :3] = syn._rot_z(0.3); P.append(T)
    p16 = init_from_eigen_batch(np.stack(P))
    n = len(P)
    dev = t["poses"].device
    poses = torch.from_numpy(p16).to(dev)
    pm = torch.zeros(n, dtype=torch.int32, device=dev)
    pl = torch.zeros(n, dtype=torch.int32, device=dev)
    tot = torch.full((n,), float(case.pose_obs_total[0]), device=dev)
    zb = core.render(poses, pm, pl).cpu().numpy()
    ref = oracle.render_depth(sc.bank.tris, sc.bank.tris_model_count, p16, np.zeros(n, np.int32),
                              np.zeros(n, np.int32), sc.width, sc.height, sc.proj, sc.src_depth_cm, sc.mask, 1.0)
    assert np.array_equal(zb, ref)
    rc, oc, df = core.evaluate(poses, pm, pl, tot, cost_type=2, stride=8)
    orc, ooc, odf = oracle.evaluate(sc.bank.tris, sc.bank.tris_model_count, p16, np.zeros(n, np.int32),
                                    np.zeros(n, np.int32), sc.width, sc.height, sc.proj, sc.src_depth_cm, sc.mask,
                                    1.0, 8, sc.cx, sc.cy, sc.fx, sc.fy, 100.0, case.obs_xyz, case.label_start,
                                    case.label_end, np.full(n, case.pose_obs_total[0], np.float32), 2, True, 0.01)
    assert _bits_equal(rc.cpu().numpy(), orc)
    assert _bits_equal(oc.cpu().numpy(), ooc)
    assert _bits_equal(df.cpu().numpy(), odf)


def _edge_pose_batch():
    P = []
    for tz in (-0.5, 0.0, 0.02, 0.05, 0.12, 0.25, 3.0):
        T = np.eye(4)
        T[:3, 3] = (0.0, 0.0, tz)
        P.append(T)
    T = np.eye(4); T[:3, 3] = (2.0, 0.0, 0.8); P.append(T)       # out of view
    T = np.eye(4); T[:3, 3] = (0.25, 0.1, 0.3); P.append(T)      # partly out of view
    T = np.eye(4); T[:3, 3] = (0.0, 0.0, 0.10); T[:3, :3] = syn._rot_z(0.3); P.append(T)
    return np.stack(P)


@pytest.mark.parametrize("tier", [0, 2, 4, 99])
def test_window_tiles_any_tier(one_object, tier, monkeypatch):
    """Pose windows ("Pose windows"): the LDS tile tier only decides which poses are scored in chunks of
    the tile.  A batch mixing ordinary and edge poses (huge / whole-image windows, poses behind
    the camera) gives the oracle's costs and z-samples with every tier, 99 being the whole image."""
    monkeypatch.setenv("PCORE_FUSED_TIER", str(tier))
    case, core, t = one_object
    sc = case.scene
    s = case.stride
    p16 = np.concatenate([case.poses[:40], init_from_eigen_batch(_edge_pose_batch()), case.poses[40:60]])
    n = len(p16)
    dev = t["poses"].device
    poses = torch.from_numpy(p16).to(dev)
    pm = torch.zeros(n, dtype=torch.int32, device=dev)
    pl = torch.zeros(n, dtype=torch.int32, device=dev)
    tot = torch.full((n,), float(case.pose_obs_total[0]), device=dev)
    hs, ws = (sc.height + s - 1) // s, sc.width // s
    dbg = torch.full((n, hs, ws), -7, dtype=torch.int32, device=dev)
    for _ in range(2):  # the second call also runs with the tier the first call's histogram picks
        rc, oc, df = core.evaluate(poses, pm, pl, tot, cost_type=2, stride=s, dbg_zs=dbg)
    orc, ooc, odf = oracle.evaluate(sc.bank.tris, sc.bank.tris_model_count, p16, np.zeros(n, np.int32),
                                    np.zeros(n, np.int32), sc.width, sc.height, sc.proj, sc.src_depth_cm, sc.mask,
                                    1.0, s, sc.cx, sc.cy, sc.fx, sc.fy, 100.0, case.obs_xyz, case.label_start,
                                    case.label_end, np.full(n, case.pose_obs_total[0], np.float32), 2, True, 0.01)
    assert _bits_equal(rc.cpu().numpy(), orc)
    assert _bits_equal(oc.cpu().numpy(), ooc)
    assert _bits_equal(df.cpu().numpy(), odf)
    full = core.render(poses, pm, pl).cpu().numpy()
    assert np.array_equal(dbg.cpu().numpy(), full[:, ::s, ::s])


def _choose_tier(hist, edge):
    """set_fused_tiles' choose_tier (pcore_api.hip): the first tier whose tile holds >= 99 % of the windows."""
    tot = sum(hist)
    over = tot
    for t, e in enumerate(edge):
        over -= hist[t]
        if e > 0 and over * 100 <= tot:
            return t
    return len(edge) - 1


def test_window_probe_picks_the_feedback_tier_on_the_first_call():
    """A fresh context has no published window histogram: its first call probes the batch's windows and starts from
    the tier that the launch's own histogram picks once published (a host running ahead of the GPU never waits for
    that feedback).  Poses pulled to half their distance (4x the window) need a tile above tier 0's; the costs are
    the oracle's whatever the tier."""
    case = SceneCase(("003_cracker_box",), n_poses=64)
    core, t = _setup(case)
    sc = case.scene
    s = case.stride
    near = case.poses.copy()
    near[:, [3, 7, 11]] *= np.float32(0.5)
    n = len(near)
    dev = t["poses"].device
    poses = torch.from_numpy(near).to(dev)
    pm = torch.zeros(n, dtype=torch.int32, device=dev)
    pl = torch.zeros(n, dtype=torch.int32, device=dev)
    tot = torch.full((n,), float(case.pose_obs_total[0]), device=dev)
    assert core.tile_info()["seq"] == -1
    rc, oc, df = core.evaluate(poses, pm, pl, tot, cost_type=2, stride=s)
    torch.cuda.synchronize()
    first = core.tile_info()
    assert first["seq"] < 1 and first["tcap"] == first["edge"][first["tier"]]  # launch 1 publishes no launch's counts
    core.evaluate(poses, pm, pl, tot, cost_type=2, stride=s)  # its workgroup 0 publishes the first launch's counts
    torch.cuda.synchronize()
    fb = core.tile_info()
    assert fb["seq"] >= 0 and sum(fb["hist"]) == n
    assert _choose_tier(fb["hist"], fb["edge"]) == first["tier"] >= 1
    orc, ooc, odf = oracle.evaluate(sc.bank.tris, sc.bank.tris_model_count, near, np.zeros(n, np.int32),
                                    np.zeros(n, np.int32), sc.width, sc.height, sc.proj, sc.src_depth_cm, sc.mask,
                                    1.0, s, sc.cx, sc.cy, sc.fx, sc.fy, 100.0, case.obs_xyz, case.label_start,
                                    case.label_end, np.full(n, case.pose_obs_total[0], np.float32), 2, True, 0.01)
    assert _bits_equal(rc.cpu().numpy(), orc)
    assert _bits_equal(oc.cpu().numpy(), ooc)
    assert _bits_equal(df.cpu().numpy(), odf)


def test_graph_replay_matches_oracle(one_object):
    """PoseCore.capture_evaluate: the captured window launch (HIP graph) re-scores new poses written in place into
    the captured tensor, with the oracle's costs, replay after replay (a captured launch publishes no tier feedback;
    the next eager call clears the counters it left)."""
    case, core, t = one_object
    sc = case.scene
    s = case.stride
    n = 32
    dev = t["poses"].device
    edge = init_from_eigen_batch(_edge_pose_batch())
    batches = [case.poses[:n], np.concatenate([edge, case.poses[40:40 + n - len(edge)]]), case.poses[n:2 * n]]
    poses = torch.from_numpy(batches[0]).to(dev).clone()
    pm = torch.zeros(n, dtype=torch.int32, device=dev)
    pl = torch.zeros(n, dtype=torch.int32, device=dev)
    tot = torch.full((n,), float(case.pose_obs_total[0]), device=dev)
    replay, (rc, oc, df) = core.capture_evaluate(poses, pm, pl, tot, cost_type=2, stride=s)
    for p16 in batches + batches[::-1]:
        poses.copy_(torch.from_numpy(p16))
        replay()
        torch.cuda.synchronize()
        orc, ooc, odf = oracle.evaluate(sc.bank.tris, sc.bank.tris_model_count, p16, np.zeros(n, np.int32),
                                        np.zeros(n, np.int32), sc.width, sc.height, sc.proj, sc.src_depth_cm,
                                        sc.mask, 1.0, s, sc.cx, sc.cy, sc.fx, sc.fy, 100.0, case.obs_xyz,
                                        case.label_start, case.label_end,
                                        np.full(n, case.pose_obs_total[0], np.float32), 2, True, 0.01)
        assert _bits_equal(rc.cpu().numpy(), orc)
        assert _bits_equal(oc.cpu().numpy(), ooc)
        assert _bits_equal(df.cpu().numpy(), odf)


def test_graph_replay_refuses_stale_context():
    """A captured evaluate graph bakes in the sampled source, the grids and the scratch pointers of its
    capture: after set_observation replay() raises instead of scoring against stale state; a fresh capture scores
    the new state correctly, and stays valid across larger eager batches."""
    from perception_amd._native import PCORE_E_STATE, PcoreError

    case = SceneCase(("003_cracker_box",), n_poses=40)
    core, t = _setup(case)
    sc = case.scene
    n = 16
    poses = t["poses"][:n].clone()
    replay, (rc, oc, df) = core.capture_evaluate(poses, t["pm"][:n], t["pl"][:n], t["tot"][:n], cost_type=2,
                                                 stride=case.stride)
    g0 = core.generation()
    replay()
    torch.cuda.synchronize()
    core.evaluate(t["poses"][:n], t["pm"][:n], t["pl"][:n], t["tot"][:n], cost_type=2, stride=case.stride)
    assert core.generation() == g0  # same-size eager calls leave the capture valid
    replay()
    # a new observation (here: the scene with its source depth shifted 5 cm back)
    src2 = t["src"] + 5
    core.set_observation(src2, t["mask"], t["obs_xyz"], t["obs_lab"], 0.01)
    with pytest.raises(PcoreError) as ei:
        replay()
    assert ei.value.code == PCORE_E_STATE
    replay2, (rc2, oc2, df2) = core.capture_evaluate(poses, t["pm"][:n], t["pl"][:n], t["tot"][:n], cost_type=2,
                                                     stride=case.stride)
    replay2()
    torch.cuda.synchronize()
    orc, ooc, odf = oracle.evaluate(sc.bank.tris, sc.bank.tris_model_count, case.poses[:n], case.pose_model[:n],
                                    case.pose_label[:n], sc.width, sc.height, sc.proj, sc.src_depth_cm + 5, sc.mask,
                                    1.0, case.stride, sc.cx, sc.cy, sc.fx, sc.fy, 100.0, case.obs_xyz,
                                    case.label_start, case.label_end, case.pose_obs_total[:n], 2, True, 0.01)
    assert _bits_equal(rc2.cpu().numpy(), orc) and _bits_equal(oc2.cpu().numpy(), ooc)
    # a larger eager batch allocates no per-batch scratch the depth-cost graph reads (since round 4 a window larger
    # than the tile is scored in chunks of it, not through an overflow list), so the capture stays valid
    big = t["poses"].repeat(64, 1)
    core.evaluate(big, t["pm"].repeat(64), t["pl"].repeat(64), t["tot"].repeat(64), cost_type=2, stride=case.stride)
    rc2.fill_(-7.0)
    replay2()
    torch.cuda.synchronize()
    assert _bits_equal(rc2.cpu().numpy(), orc) and _bits_equal(oc2.cpu().numpy(), ooc)
    core.close()


def test_evaluate_icp_invalid_call_writes_nothing(one_object):
    """evaluate_icp validates everything the final re-score checks before its first chunk runs: a call with
    calc_obs_cost and no observed-cost outputs fails with INVALID_ARG and leaves the adjusted poses
    untouched; an image whose sampled z-buffer cannot fit in LDS is INVALID_ARG too, not a failed launch."""
    import ctypes

    from perception_amd import _native
    from perception_amd._native import EvalParams, IcpParams, PcoreError

    case, core, t = one_object
    n = 8
    dev = t["poses"].device
    adj = torch.full((n, 16), -7.0, device=dev)
    rc = torch.full((n,), -7.0, device=dev)
    p = EvalParams(2, 1, case.stride, 100.0, 0.01, 1.0, 15.0)
    ip = IcpParams(_native.ICP_K, _native.ICP_MAX_ITER, _native.ICP_ROT_EPS, _native.ICP_TRANS_EPS)
    vp = ctypes.c_void_p
    r = core.lib.pcore_evaluate_icp(core._h, vp(t["poses"].data_ptr()), vp(t["pm"].data_ptr()),
                                    vp(t["pl"].data_ptr()), vp(t["tot"].data_ptr()), n, ctypes.byref(p),
                                    ctypes.byref(ip), vp(adj.data_ptr()), None, vp(rc.data_ptr()), None, None,
                                    vp(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert r == _native.PCORE_E_INVALID_ARG
    assert (adj == -7.0).all() and (rc == -7.0).all()
    with pytest.raises(PcoreError) as ei:
        core.evaluate_icp(t["poses"][:n], t["pm"][:n], t["pl"][:n], t["tot"][:n], cost_type=2, stride=1)
    assert ei.value.code == _native.PCORE_E_INVALID_ARG


def test_evaluate_icp_multi_chunk_equals_single_chunk(monkeypatch):
    """The GICP scratch budget splits a batch into equal chunks (pose_base offsets, per-chunk queue order):
    4,000 C2 poses under a 1 GiB budget (3,495 poses per chunk at 640x480 / stride 8) run as two chunks and
    give the single-chunk result bit for bit (adjusted poses, iterations, costs)."""
    from perception_amd import workloads

    w = workloads.build(poses_per_model=4000)
    one = [x.cpu().numpy() for x in w.core.evaluate_icp(w.poses, w.pose_model, w.pose_label, w.pose_obs_total,
                                                          stride=w.stride)]
    monkeypatch.setenv("PCORE_ICP_SCRATCH_GIB", "1")
    two = [x.cpu().numpy() for x in w.core.evaluate_icp(w.poses, w.pose_model, w.pose_label, w.pose_obs_total,
                                                          stride=w.stride)]
    for a, b in zip(one, two):
        assert _bits_equal(a, b)
    assert one[1].max() == 150 and (one[0] != w.poses.cpu().numpy()).any()


def test_empty_batch_and_errors(one_object):
    case, core, t = one_object
    dev = t["poses"].device
    e = torch.empty((0, 16), dtype=torch.float32, device=dev)
    ei = torch.empty((0,), dtype=torch.int32, device=dev)
    ef = torch.empty((0,), dtype=torch.float32, device=dev)
    rc, oc, df = core.evaluate(e, ei, ei, ef, cost_type=2, stride=8)
    assert rc.numel() == 0
    from perception_amd._native import PcoreError
    with pytest.raises(PcoreError):
        core.evaluate(t["poses"][:2], t["pm"][:2], t["pl"][:2], t["tot"][:2], cost_type=1, stride=8)
    with pytest.raises(PcoreError):
        core.evaluate(t["poses"][:2], t["pm"][:2], t["pl"][:2], t["tot"][:2], cost_type=2, stride=7)


@pytest.mark.parametrize("name", ["oracle_scene_1obj.npz", "oracle_scene_3obj.npz"])
def test_gpu_reproduces_committed_fixture(name):
    import hashlib
    import os

    g = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name)))
    W, H = int(g["cam"][0]), int(g["cam"][1])
    fx, fy, cx, cy = (float(v) for v in g["cam"][2:])
    stride = int(g["stride"])
    K = len(g["tris_model_count"])
    dev = torch.device("cuda", 0)
    core = PoseCore(0)
    core.upload_meshes(g["tris"], g["tris_model_count"])
    core.set_camera(W, H, fx, fy, cx, cy, g["proj"])
    mask = torch.from_numpy(g["mask"]).to(dev)
    xyz, lab = core.observed_cloud(torch.from_numpy(g["depth_raw"]).to(dev), mask, stride, float(g["depth_factor"]))
    assert _bits_equal(xyz.cpu().numpy(), g["obs_xyz"]) and np.array_equal(lab.cpu().numpy(), g["obs_label"])
    core.set_observation(torch.from_numpy(g["src_depth_cm"]).to(dev), mask, xyz, lab, 0.01)
    poses = torch.from_numpy(g["poses"]).to(dev)
    pm = torch.from_numpy(g["pose_model"]).to(dev)
    z = core.render(poses, pm, pm).cpu().numpy()
    assert [hashlib.sha256(np.ascontiguousarray(zi).tobytes()).hexdigest() for zi in z] == list(g["z_hash"])
    rc, oc, df = core.evaluate(poses, pm, pm, torch.from_numpy(g["pose_obs_total"]).to(dev), cost_type=2,
                               stride=stride)
    assert _bits_equal(rc.cpu().numpy(), g["rc"])
    assert _bits_equal(oc.cpu().numpy(), g["oc"])
    assert _bits_equal(df.cpu().numpy(), g["diff"])
    cost, idx = decode_keys(core.select(rc, oc, pm, K))
    assert np.array_equal(cost, g["best_cost"]) and np.array_equal(idx, g["best_index"])


def _label_covs(case, six=True):
    cov = np.zeros((len(case.obs_xyz), 6))
    if six:
        for L in range(len(case.label_start)):
            a, b = case.label_start[L], case.label_end[L]
            if b > a:
                cov[a:b] = oracle.covariances(case.obs_xyz[a:b])
    else:
        cov = oracle.covariances(case.obs_xyz)
    return cov


@pytest.mark.parametrize("kernel", ["narrow", "wide"])
@pytest.mark.parametrize("fixture", ["one_object", "three_objects"])
def test_evaluate_icp_matches_oracle(fixture, kernel, request, monkeypatch):
    """Both GICP kernels -- one wave per pose (large batches) and eight waves per pose (small batches) --
    against the oracle; PCORE_GICP_KERNEL pins the choice launch_gicp otherwise makes by batch size."""
    case, core, t = request.getfixturevalue(fixture)
    sc = case.scene
    n = min(48, len(case.poses))
    monkeypatch.setenv("PCORE_GICP_KERNEL", kernel)
    adj, iters, rc, oc, df = core.evaluate_icp(t["poses"][:n], t["pm"][:n], t["pl"][:n], t["tot"][:n],
                                               cost_type=2, stride=case.stride)
    oadj, oit, orc, ooc, odf = oracle.evaluate_icp(
        sc.bank.tris, sc.bank.tris_model_count, case.poses[:n], case.pose_model[:n], case.pose_label[:n],
        sc.width, sc.height, sc.proj, sc.src_depth_cm, sc.mask, 1.0, case.stride, sc.cx, sc.cy, sc.fx, sc.fy,
        100.0, case.obs_xyz, _label_covs(case), case.label_start, case.label_end, case.pose_obs_total[:n], 2, True,
        0.01)
    adj = adj.cpu().numpy()
    # GICP transform within 1e-4 (north_star); the build-owned spec is in fact bit-reproducible
    assert np.abs(adj - oadj).max() <= 1e-4 * 100, np.abs(adj - oadj).max()
    assert np.array_equal(iters.cpu().numpy(), oit)
    assert _bits_equal(adj, oadj)
    assert _bits_equal(rc.cpu().numpy(), orc)
    assert _bits_equal(oc.cpu().numpy(), ooc)
    assert _bits_equal(df.cpu().numpy(), odf)


@pytest.mark.parametrize("kernel", ["narrow", "wide"])
def test_evaluate_icp_edge_poses_match_oracle(one_object, kernel, monkeypatch):
    """GICP on the edge-pose batch: empty source clouds (behind the camera, out of view), clouds of a few points
    (fewer than k = 10 neighbours), and poses so close that the cloud fills most of the sampled image -- more points
    than the correspondence history holds and than the trials keep in LDS, so those poses search every iteration and
    read their later rounds' trial inputs from scratch.  Iterations, refined poses and costs bit for bit."""
    case, core, t = one_object
    sc = case.scene
    p16 = init_from_eigen_batch(_edge_pose_batch())
    n = len(p16)
    dev = t["poses"].device
    poses = torch.from_numpy(p16).to(dev)
    pm = torch.zeros(n, dtype=torch.int32, device=dev)
    pl = torch.zeros(n, dtype=torch.int32, device=dev)
    tot_h = np.full(n, case.pose_obs_total[0], np.float32)
    tot = torch.from_numpy(tot_h).to(dev)
    monkeypatch.setenv("PCORE_GICP_KERNEL", kernel)
    adj, iters, rc, oc, df = core.evaluate_icp(poses, pm, pl, tot, cost_type=2, stride=case.stride)
    z = np.zeros(n, np.int32)
    oadj, oit, orc, ooc, odf = oracle.evaluate_icp(
        sc.bank.tris, sc.bank.tris_model_count, p16, z, z, sc.width, sc.height, sc.proj, sc.src_depth_cm, sc.mask,
        1.0, case.stride, sc.cx, sc.cy, sc.fx, sc.fy, 100.0, case.obs_xyz, _label_covs(case), case.label_start,
        case.label_end, tot_h, 2, True, 0.01)
    counts = [len(oracle.depth_to_cloud(d, case.stride, sc.cx, sc.cy, sc.fx, sc.fy, 100.0)[0])
              for d in oracle.render_depth(sc.bank.tris, sc.bank.tris_model_count, p16, z, z, sc.width, sc.height,
                                           sc.proj, sc.src_depth_cm, sc.mask, 1.0)]
    # the batch covers the cases named above: empty, fewer than k points, more than kCorrHistCap (512) points
    assert min(counts) == 0 and any(0 < c < 10 for c in counts) and max(counts) > 512, counts
    assert np.array_equal(iters.cpu().numpy(), oit)
    assert _bits_equal(adj.cpu().numpy(), oadj)
    assert _bits_equal(rc.cpu().numpy(), orc)
    assert _bits_equal(oc.cpu().numpy(), ooc)
    assert _bits_equal(df.cpu().numpy(), odf)


def test_evaluate_icp_chunked_cloud_tile_matches_oracle(three_objects, monkeypatch):
    """With a 64-sample tile the GICP source clouds are rastered in chunks of the tile (render_cloud_kernel's row
    bands / column blocks) and appended chunk after chunk: the reference's row-major compaction order, so the refined
    poses and costs stay the oracle's bit for bit."""
    case, core, t = three_objects
    sc = case.scene
    n = min(32, len(case.poses))
    monkeypatch.setenv("PCORE_FUSED_TCAP", "64")
    adj, iters, rc, oc, df = core.evaluate_icp(t["poses"][:n], t["pm"][:n], t["pl"][:n], t["tot"][:n],
                                               cost_type=2, stride=case.stride)
    oadj, oit, orc, ooc, odf = oracle.evaluate_icp(
        sc.bank.tris, sc.bank.tris_model_count, case.poses[:n], case.pose_model[:n], case.pose_label[:n],
        sc.width, sc.height, sc.proj, sc.src_depth_cm, sc.mask, 1.0, case.stride, sc.cx, sc.cy, sc.fx, sc.fy,
        100.0, case.obs_xyz, _label_covs(case), case.label_start, case.label_end, case.pose_obs_total[:n], 2, True,
        0.01)
    assert np.array_equal(iters.cpu().numpy(), oit)
    assert _bits_equal(adj.cpu().numpy(), oadj)
    assert _bits_equal(rc.cpu().numpy(), orc)
    assert _bits_equal(oc.cpu().numpy(), ooc)
    assert _bits_equal(df.cpu().numpy(), odf)


def test_evaluate_icp_3dof_matches_oracle(one_object):
    case, core, t = one_object
    sc = case.scene
    n = 24
    tot = np.full(n, len(case.obs_xyz), np.float32)
    adj, iters, rc, oc, df = core.evaluate_icp(t["poses"][:n], t["pm"][:n], None,
                                               torch.from_numpy(tot).to(t["poses"].device), cost_type=0,
                                               stride=case.stride)
    oadj, oit, orc, ooc, odf = oracle.evaluate_icp(
        sc.bank.tris, sc.bank.tris_model_count, case.poses[:n], case.pose_model[:n], None, sc.width, sc.height,
        sc.proj, sc.src_depth_cm, None, 1.0, case.stride, sc.cx, sc.cy, sc.fx, sc.fy, 100.0, case.obs_xyz,
        _label_covs(case, six=False), None, None, tot, 0, True, 0.01)
    assert np.array_equal(iters.cpu().numpy(), oit)
    assert _bits_equal(adj.cpu().numpy(), oadj)
    assert _bits_equal(rc.cpu().numpy(), orc)


@pytest.mark.parametrize("obs_stride", [2, 1])
def test_evaluate_icp_dense_targets_matches_oracle(one_object, obs_stride):
    """Observed cloud at stride 2 / 1 (label segments of ~2k / ~8k points): the target tiling paths of the
    GICP and covariance kernels."""
    case, core, t = one_object
    sc = case.scene
    xyz, lab = core.observed_cloud(t["raw"], t["mask"], obs_stride, sc.depth_factor)
    oxyz, _, olab = oracle.depth_to_cloud(sc.depth_raw, obs_stride, sc.cx, sc.cy, sc.fx, sc.fy, sc.depth_factor,
                                          label_mask=sc.mask)
    assert _bits_equal(xyz.cpu().numpy(), oxyz) and np.array_equal(lab.cpu().numpy(), olab)
    order = np.argsort(olab, kind="stable")
    oxyz, olab = oxyz[order], olab[order]
    ls = np.array([np.searchsorted(olab, L, "left") for L in range(case.K)], np.int32)
    le = np.array([np.searchsorted(olab, L, "right") for L in range(case.K)], np.int32)
    assert (le - ls).max() > 1024
    tot = (le - ls).astype(np.float32)[case.pose_label]
    ocov = np.zeros((len(oxyz), 6))
    for L in range(case.K):
        ocov[ls[L]:le[L]] = oracle.covariances(oxyz[ls[L]:le[L]])
    n = 16
    try:
        core.set_observation(t["src"], t["mask"], xyz, lab, 0.01)
        adj, iters, rc, oc, df = core.evaluate_icp(t["poses"][:n], t["pm"][:n], t["pl"][:n],
                                                   torch.from_numpy(tot[:n]).to(t["poses"].device),
                                                   cost_type=2, stride=case.stride)
    finally:
        core.set_observation(t["src"], t["mask"], t["obs_xyz"], t["obs_lab"], 0.01)
    oadj, oit, orc, ooc, odf = oracle.evaluate_icp(
        sc.bank.tris, sc.bank.tris_model_count, case.poses[:n], case.pose_model[:n], case.pose_label[:n],
        sc.width, sc.height, sc.proj, sc.src_depth_cm, sc.mask, 1.0, case.stride, sc.cx, sc.cy, sc.fx, sc.fy,
        100.0, oxyz, ocov, ls, le, tot[:n], 2, True, 0.01)
    assert np.array_equal(iters.cpu().numpy(), oit)
    assert _bits_equal(adj.cpu().numpy(), oadj)
    assert _bits_equal(rc.cpu().numpy(), orc)
    assert _bits_equal(oc.cpu().numpy(), ooc)


def test_evaluate_icp_tied_and_near_zero_keys_matches_oracle(three_objects):
    """Correspondence ties across key quads and keys near zero: every label segment gets exact
    copies of every third of its points appended after it (equal distances at indices in other quads: the first
    index must win), one point at the segment's key origin and one a float ulp away from another point.  GICP
    poses, iteration counts and costs bit-exact vs the oracle."""
    case, core, t = three_objects
    sc = case.scene
    xyz = case.obs_xyz_raw.astype(np.float32)
    lab = case.obs_label_raw.astype(np.int32)
    extra_p, extra_l = [], []
    for L in range(case.K):
        seg = xyz[lab == L]
        if len(seg) == 0:
            continue
        lo, hi = seg.min(0), seg.max(0)
        origin = ((lo + hi) * np.float32(0.5)).astype(np.float32)  # the key origin: t' = 0, key = 0 exactly
        near = seg[0].copy()
        near[0] = np.nextafter(near[0], np.float32(np.inf))
        add = np.concatenate([seg[::3], origin[None], near[None]])
        extra_p.append(add)
        extra_l.append(np.full(len(add), L, np.int32))
    xyz2 = np.concatenate([xyz] + extra_p).astype(np.float32)
    lab2 = np.concatenate([lab] + extra_l)
    order = np.argsort(lab2, kind="stable")
    oxyz, olab = xyz2[order], lab2[order]
    ls = np.array([np.searchsorted(olab, L, "left") for L in range(case.K)], np.int32)
    le = np.array([np.searchsorted(olab, L, "right") for L in range(case.K)], np.int32)
    tot = (le - ls).astype(np.float32)[case.pose_label]
    ocov = np.zeros((len(oxyz), 6))
    for L in range(case.K):
        ocov[ls[L]:le[L]] = oracle.covariances(oxyz[ls[L]:le[L]])
    n = 24
    dev = t["poses"].device
    try:
        core.set_observation(t["src"], t["mask"], torch.from_numpy(xyz2).to(dev), torch.from_numpy(lab2).to(dev),
                             0.01)
        adj, iters, rc, oc, df = core.evaluate_icp(t["poses"][:n], t["pm"][:n], t["pl"][:n],
                                                   torch.from_numpy(tot[:n]).to(dev), cost_type=2,
                                                   stride=case.stride)
    finally:
        core.set_observation(t["src"], t["mask"], t["obs_xyz"], t["obs_lab"], 0.01)
    oadj, oit, orc, ooc, odf = oracle.evaluate_icp(
        sc.bank.tris, sc.bank.tris_model_count, case.poses[:n], case.pose_model[:n], case.pose_label[:n],
        sc.width, sc.height, sc.proj, sc.src_depth_cm, sc.mask, 1.0, case.stride, sc.cx, sc.cy, sc.fx, sc.fy,
        100.0, oxyz, ocov, ls, le, tot[:n], 2, True, 0.01)
    assert np.array_equal(iters.cpu().numpy(), oit)
    assert _bits_equal(adj.cpu().numpy(), oadj)
    assert _bits_equal(rc.cpu().numpy(), orc)
    assert _bits_equal(oc.cpu().numpy(), ooc)


def test_observed_cloud_bounded_matches_oracle(one_object):
    """3-DoF depth2cloud_global: world-frame table bounds filter and colours (f4)."""
    case, core, t = one_object
    sc = case.scene
    rng = np.random.default_rng(11)
    rgb = rng.integers(0, 256, (sc.height, sc.width, 3), dtype=np.uint8)
    cam_to_world = np.array([[0, 0, 1, 0.1], [-1, 0, 0, 0.2], [0, -1, 0, 0.9], [0, 0, 0, 1]], np.float32)
    dev = t["raw"].device
    for stride in (8, 4):
        for bounds in (None, [1.0, 0.0, 0.3, -0.3, 1.2, 0.5], [0.9, 0.8, 0.2, 0.1, 1.0, 0.85]):
            M = None if bounds is None else cam_to_world
            xyz, col = core.observed_cloud_bounded(t["raw"], stride, sc.depth_factor, M, bounds,
                                                   rgb=torch.from_numpy(rgb).to(dev))
            oxyz, ocol = oracle.depth_to_cloud_bounded(sc.depth_raw, stride, sc.cx, sc.cy, sc.fx, sc.fy,
                                                       sc.depth_factor, M, bounds, rgb)
            assert len(oxyz) > 0
            assert _bits_equal(xyz.cpu().numpy(), oxyz)
            assert np.array_equal(col.cpu().numpy(), ocol)
    # without bounds the point set equals pcore_observed_cloud without a mask
    xyz, _ = core.observed_cloud_bounded(t["raw"], 8, sc.depth_factor)
    ref, _ = core.observed_cloud(t["raw"], None, 8, sc.depth_factor)
    assert torch.equal(xyz, ref)


@pytest.mark.parametrize("kernel", ["narrow", "wide"])
def test_evaluate_icp_3dof_whole_scene_targets_matches_oracle(kernel, monkeypatch):
    """C1's table-top scene with the WHOLE observed cloud as the GICP target (~19k points at stride 4, no
    labels): correspondences and target covariances take the exact grid shell search; the result must equal
    the oracle's brute-force scans bit for bit."""
    from perception_amd import workloads
    from tests.helpers import oracle_render_fn
    c1 = workloads.c1_tabletop(oracle_render_fn)
    sc = c1.scene
    core = PoseCore(0)
    core.upload_meshes(sc.bank.tris, sc.bank.tris_model_count)
    core.set_camera(sc.width, sc.height, sc.fx, sc.fy, sc.cx, sc.cy, sc.proj)
    dev = torch.device("cuda", 0)
    xyz, _ = core.observed_cloud_bounded(torch.from_numpy(sc.depth_raw).to(dev), 4, sc.depth_factor)
    assert xyz.shape[0] > 4 * 2048
    core.set_observation(torch.from_numpy(c1.src_depth_cm).to(dev), None, xyz, None, 0.0075)
    idx = np.array([c1.gt_index, 3, 70], np.int64)
    n = len(idx)
    monkeypatch.setenv("PCORE_GICP_KERNEL", kernel)
    poses = c1.poses[idx]
    tot = np.full(n, xyz.shape[0], np.float32)
    adj, iters, rc, oc, df = core.evaluate_icp(torch.from_numpy(poses).to(dev), torch.zeros(n, dtype=torch.int32,
                                               device=dev), None, torch.from_numpy(tot).to(dev), cost_type=0,
                                               stride=4, sensor_resolution=0.0075)
    oxyz = xyz.cpu().numpy()
    ocov = oracle.covariances(oxyz)
    oadj, oit, orc, ooc, odf = oracle.evaluate_icp(
        sc.bank.tris, sc.bank.tris_model_count, poses, np.zeros(n, np.int32), None, sc.width, sc.height, sc.proj,
        c1.src_depth_cm, None, 1.0, 4, sc.cx, sc.cy, sc.fx, sc.fy, 100.0, oxyz, ocov, None, None, tot, 0, True,
        0.0075)
    assert np.array_equal(iters.cpu().numpy(), oit)
    assert _bits_equal(adj.cpu().numpy(), oadj)
    assert _bits_equal(rc.cpu().numpy(), orc)
    assert _bits_equal(oc.cpu().numpy(), ooc)


@pytest.mark.parametrize("kernel", ["narrow", "wide"])
def test_evaluate_icp_3dof_far_queries_match_oracle(kernel, monkeypatch):
    """C1's poses that GICP walks away from the scene (the most iterations of the 128): their queries end far from
    every point of the 19.2 k-point whole-scene target, where the shell search runs past its 343-cell minimum (the
    budget scales with the segment) or falls back to the in-order scan.  Adjusted poses, iteration counts and costs
    bit-exact vs the oracle's brute force."""
    from perception_amd import workloads
    from tests.helpers import oracle_render_fn
    c1 = workloads.c1_tabletop(oracle_render_fn)
    sc = c1.scene
    core = PoseCore(0)
    core.upload_meshes(sc.bank.tris, sc.bank.tris_model_count)
    core.set_camera(sc.width, sc.height, sc.fx, sc.fy, sc.cx, sc.cy, sc.proj)
    dev = torch.device("cuda", 0)
    xyz, _ = core.observed_cloud_bounded(torch.from_numpy(sc.depth_raw).to(dev), 4, sc.depth_factor)
    core.set_observation(torch.from_numpy(c1.src_depth_cm).to(dev), None, xyz, None, 0.0075)
    monkeypatch.setenv("PCORE_GICP_KERNEL", kernel)
    n_all = len(c1.poses)
    tot_all = torch.full((n_all,), float(xyz.shape[0]), dtype=torch.float32, device=dev)
    _, it_all, _, _, _ = core.evaluate_icp(torch.from_numpy(c1.poses).to(dev), torch.zeros(n_all, dtype=torch.int32,
                                           device=dev), None, tot_all, cost_type=0, stride=4, sensor_resolution=0.0075)
    it_all = it_all.cpu().numpy()
    idx = np.argsort(-it_all, kind="stable")[:2]
    assert it_all[idx].min() >= 100, it_all[idx]
    n = len(idx)
    poses = c1.poses[idx]
    tot = np.full(n, xyz.shape[0], np.float32)
    adj, iters, rc, oc, df = core.evaluate_icp(torch.from_numpy(poses).to(dev), torch.zeros(n, dtype=torch.int32,
                                               device=dev), None, torch.from_numpy(tot).to(dev), cost_type=0,
                                               stride=4, sensor_resolution=0.0075)
    assert np.array_equal(iters.cpu().numpy(), it_all[idx])  # batch-invariant
    oxyz = xyz.cpu().numpy()
    ocov = oracle.covariances(oxyz)
    oadj, oit, orc, ooc, odf = oracle.evaluate_icp(
        sc.bank.tris, sc.bank.tris_model_count, poses, np.zeros(n, np.int32), None, sc.width, sc.height, sc.proj,
        c1.src_depth_cm, None, 1.0, 4, sc.cx, sc.cy, sc.fx, sc.fy, 100.0, oxyz, ocov, None, None, tot, 0, True,
        0.0075)
    assert np.array_equal(iters.cpu().numpy(), oit)
    assert _bits_equal(adj.cpu().numpy(), oadj)
    assert _bits_equal(rc.cpu().numpy(), orc)
    assert _bits_equal(oc.cpu().numpy(), ooc)


def test_pose_lanes_overlapped_batches_match_oracle(three_objects):
    """core.PoseLanes (the bench's two batches in flight): batches submitted round-robin to two contexts on two
    streams, with no synchronisation between them, each give the oracle's costs bit for bit."""
    from perception_amd.core import PoseLanes

    case, core, t = three_objects
    sc = case.scene

    def setup(c):
        c.upload_meshes(sc.bank.tris, sc.bank.tris_model_count)
        c.set_camera(sc.width, sc.height, sc.fx, sc.fy, sc.cx, sc.cy, sc.proj)
        c.set_observation(t["src"], t["mask"], t["obs_xyz"], t["obs_lab"], 0.01)

    lanes = PoseLanes(0, 2)
    for c in lanes.cores:
        setup(c)
    torch.cuda.synchronize()
    n = len(case.poses)
    outs = []
    for i in range(6):  # six batches, three per lane, back to back
        c, st = lanes[i % 2]
        with torch.cuda.stream(st):
            outs.append(c.evaluate(t["poses"], t["pm"], t["pl"], t["tot"], cost_type=2, stride=case.stride,
                                   stream=st))
    torch.cuda.synchronize()
    orc, ooc, odf = case.oracle_costs(cost_type=2)
    for rc, oc, df in outs:
        assert rc.shape[0] == n
        assert np.array_equal(rc.cpu().numpy(), orc) and np.array_equal(oc.cpu().numpy(), ooc)
        assert np.array_equal(df.cpu().numpy(), odf)


def test_general_projection_matrix(one_object):
    """A projection without compute_proj's zeros (skew and offsets in rows 0 / 1) takes the full four-term
    rows in the fused kernel's vertex pass: its sampled z-buffers equal the oracle's full render, and the
    sparse-row path of the default camera is not taken."""
    case, _, t = one_object
    sc = case.scene
    proj = sc.proj.copy()
    proj[1], proj[3], proj[4], proj[7] = np.float32(0.0123), np.float32(0.0625), np.float32(-0.0071), np.float32(-0.03)
    core = PoseCore(0)
    core.upload_meshes(sc.bank.tris, sc.bank.tris_model_count)
    core.set_camera(sc.width, sc.height, sc.fx, sc.fy, sc.cx, sc.cy, proj)
    core.set_observation(t["src"], t["mask"], t["obs_xyz"], t["obs_lab"], 0.01)
    n, s = 32, case.stride
    hs, ws = (sc.height + s - 1) // s, sc.width // s
    dbg = torch.empty((n, hs, ws), dtype=torch.int32, device=t["poses"].device)
    core.evaluate(t["poses"][:n], t["pm"][:n], t["pl"][:n], t["tot"][:n], cost_type=2, stride=s, dbg_zs=dbg)
    ref = oracle.render_depth(sc.bank.tris, sc.bank.tris_model_count, case.poses[:n], case.pose_model[:n],
                              case.pose_label[:n], sc.width, sc.height, proj, sc.src_depth_cm, sc.mask, 1.0)
    assert (ref > 0).sum() > 0
    assert np.array_equal(dbg.cpu().numpy(), ref[:, ::s, ::s])


@pytest.mark.parametrize("labels", [True, False])
def test_render_color_planes_bit_exact(labels):
    """Stage RENDER / DEBUG colour planes (renderer.cu:1594-1615): the reference's result_color -- red, green and
    blue planes of N x H x W -- against the oracle's serial z-test with colour writes and black-out
    (image_renderer.cuh:146-196), per-triangle colours random so every tie and occlusion shows."""
    case = SceneCase(("003_cracker_box", "005_tomato_soup_can", "061_foam_brick"), n_poses=8, seed=5)
    sc = case.scene
    rng = np.random.default_rng(9)
    rgb = rng.integers(0, 256, size=(len(sc.bank.tris), 3), dtype=np.uint8)
    core = PoseCore(0)
    core.upload_meshes(sc.bank.tris, sc.bank.tris_model_count, colors=rgb)
    core.set_camera(sc.width, sc.height, sc.fx, sc.fy, sc.cx, sc.cy, sc.proj)
    dev = torch.device("cuda", 0)
    raw, mask = torch.from_numpy(sc.depth_raw).to(dev), torch.from_numpy(sc.mask).to(dev)
    xyz, lab = core.observed_cloud(raw, mask, 8, sc.depth_factor)
    core.set_observation(torch.from_numpy(sc.src_depth_cm).to(dev), mask, xyz, lab, 0.01)
    poses = torch.from_numpy(case.poses).to(dev)
    pm = torch.from_numpy(case.pose_model).to(dev)
    pl = torch.from_numpy(case.pose_label).to(dev) if labels else None
    zb, col = core.render(poses, pm, pl, color=True)
    rz, rc = oracle.render_depth_color(sc.bank.tris, rgb, sc.bank.tris_model_count, case.poses, case.pose_model,
                                       case.pose_label if labels else None, sc.width, sc.height, sc.proj,
                                       sc.src_depth_cm, sc.mask if labels else None, 1.0)
    assert np.array_equal(zb.cpu().numpy(), rz)
    got = col.cpu().numpy()
    assert got.shape == rc.shape == (3, len(case.poses), sc.height, sc.width)
    mism = np.argwhere(got != rc)
    assert len(mism) == 0, f"{len(mism)} mismatching colour samples, first {mism[:5]}"
    assert (rc.max(0) > 0).sum() > 1000
    # the depth-only call is unchanged by the colour pass
    assert np.array_equal(core.render(poses, pm, pl).cpu().numpy(), rz)
