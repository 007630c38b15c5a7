"""Benchmark / smoke workloads (BASELINE.json configs) built on the GPU path.

C2: single YCB mesh (003_cracker_box proxy, 12,288 triangles), 10k 6-DoF candidate poses rendered and
scored at 640x480, stride 8, no ICP.  The observed scene is the GPU RENDER stage of a GT pose, turned
into 16-bit depth (depth_factor 10000, N(0, 2 mm) noise), a background plane and a label mask, then
unprojected with depth2cloud_global on the GPU.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Sequence

import numpy as np
import torch

from . import synthetic as syn
from ._native import COST_DEPTH_6DOF
from .core import PoseCore
from .model import init_from_eigen_batch


@dataclass
class Workload:
    core: PoseCore
    scene: syn.Scene
    poses: torch.Tensor          # (N, 16) f32
    pose_model: torch.Tensor     # (N,) i32
    pose_label: torch.Tensor     # (N,) i32
    pose_obs_total: torch.Tensor  # (N,) f32
    obs_xyz: torch.Tensor
    obs_label: torch.Tensor
    stride: int
    index_base: int
    num_models: int
    gt_index: Sequence[int]


def object_centers(K: int):
    """K object centres on a grid in front of the camera (0.7-1.2 m), well inside the 640x480 view.

    More than 9 objects (C4's 21-model bank) go on a 7-column grid at 1.05 m: on the square grid with
    depths alternating over 0.75 / 0.975 / 1.2 m, 040_large_marker sat behind 024_bowl and had no
    visible sample, so its model could not be found.  On this grid every object keeps >= 94 % of its
    unoccluded stride-8 samples (tests/test_host.py::test_c4_scene_every_object_visible)."""
    if K == 1:
        return [(0.03, -0.02, 0.80)]
    if K > 9:
        cols = 7
        rows = int(np.ceil(K / cols))
        return [(-0.48 + 0.96 * (i % cols) / (cols - 1), -0.26 + 0.52 * (i // cols) / max(rows - 1, 1), 1.05)
                for i in range(K)]
    cols = int(np.ceil(np.sqrt(K)))
    rows = int(np.ceil(K / cols))
    out = []
    for i in range(K):
        r, c = divmod(i, cols)
        x = -0.30 + 0.60 * (c / max(cols - 1, 1))
        y = -0.20 + 0.40 * (r / max(rows - 1, 1))
        out.append((x, y, 0.75 + 0.45 * (i % 3) / 2))
    return out


def gpu_render_fn(core: PoseCore, device):
    def fn(tris, cnt, p16, pm, W, H, proj):
        poses = torch.from_numpy(np.ascontiguousarray(p16)).to(device)
        pmt = torch.from_numpy(np.ascontiguousarray(pm, dtype=np.int32)).to(device)
        return core.render(poses, pmt, None).cpu().numpy()
    return fn


def build(names: Sequence[str] = ("003_cracker_box",), poses_per_model: int = 10000, cam: dict = syn.CAM_640,
          stride: int = 8, device: int = 0, rank: int = 0, seed: int = syn.SEED, k: int = 32) -> Workload:
    dev = torch.device("cuda", device)
    rng = np.random.default_rng(seed)
    K = len(names)
    bank = syn.model_bank(names, k)
    core = PoseCore(device)
    core.upload_meshes(bank.tris, bank.tris_model_count, bank.colors)
    from .model import compute_proj
    proj = compute_proj(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["width"], cam["height"])
    core.set_camera(cam["width"], cam["height"], cam["fx"], cam["fy"], cam["cx"], cam["cy"], proj)
    # empty observation (no source occlusion) to render the GT scene
    W, H = cam["width"], cam["height"]
    zero = torch.zeros((H, W), dtype=torch.int32, device=dev)
    core.set_observation(zero, None, torch.zeros((0, 3), dtype=torch.float32, device=dev), None, 0.01)
    centers = object_centers(K)
    gts = np.stack([syn.default_gt_pose(rng, c) for c in centers])
    scene = syn.make_scene(list(names), gts, gpu_render_fn(core, dev), cam=cam, rng=rng, k=k)
    raw = torch.from_numpy(scene.depth_raw).to(dev)
    mask = torch.from_numpy(scene.mask).to(dev)
    obs_xyz, obs_label = core.observed_cloud(raw, mask, stride, scene.depth_factor)
    core.set_observation(torch.from_numpy(scene.src_depth_cm).to(dev), mask, obs_xyz, obs_label, 0.01)
    seg = np.bincount(obs_label.cpu().numpy(), minlength=K).astype(np.float32)
    poses, models, gt_index = [], [], []
    prng = np.random.default_rng(seed + 1 + rank)
    for obj in range(K):
        P = syn.candidate_poses(gts[obj][:3, 3], poses_per_model, prng, include=gts[obj])
        gt_index.append(sum(len(p) for p in poses) + poses_per_model // 3)
        poses.append(P)
        models.append(np.full(len(P), obj, np.int32))
    p16 = init_from_eigen_batch(np.concatenate(poses))
    pm = np.concatenate(models)
    n = len(pm)
    return Workload(core, scene, torch.from_numpy(p16).to(dev), torch.from_numpy(pm).to(dev),
                    torch.from_numpy(pm.copy()).to(dev), torch.from_numpy(seg[pm]).to(dev), obs_xyz, obs_label,
                    stride, rank * n, K, gt_index)


def lanes(w: Workload, count: int = 2):
    """core.PoseLanes over the workload's context plus count - 1 more with the same meshes, camera and
    observation (the bench keeps two batches in flight)."""
    from .core import PoseLanes

    sc = w.scene
    dev = w.poses.device
    src = torch.from_numpy(sc.src_depth_cm).to(dev)
    mask = torch.from_numpy(sc.mask).to(dev)

    def setup(c):
        c.upload_meshes(sc.bank.tris, sc.bank.tris_model_count, sc.bank.colors)
        c.set_camera(sc.width, sc.height, sc.fx, sc.fy, sc.cx, sc.cy, sc.proj)
        c.set_observation(src, mask, w.obs_xyz, w.obs_label, 0.01)

    ln = PoseLanes.replicate(w.core, setup, count)
    torch.cuda.synchronize(dev)
    return ln


def step(w: Workload, out, keys):
    """One pass of the hot path over the batch: render + score every pose, fold the argmin keys."""
    rc, oc, df = w.core.evaluate(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, cost_type=COST_DEPTH_6DOF,
                                 stride=w.stride, out=out)
    w.core.select(rc, oc, w.pose_model, w.num_models, index_base=w.index_base, keys=keys)
    return rc, oc, df


@dataclass
class C1Workload:
    """BASELINE.json configs[0]: one 003_cracker_box proxy, 128 3-DoF poses (4 x 4 x 8 yaw steps of pi/4 on
    the table plane, the ground truth among them) at 640x480."""
    scene: "syn.TabletopScene"
    poses: np.ndarray          # (128, 16) f32 cm-scaled mat4x4, camera frame
    states: np.ndarray         # (128, 3) x, y, yaw in the world
    gt_index: int
    src_depth_cm: np.ndarray   # (H, W) int32 cm (search_env.cpp:2487-2498)


def c1_tabletop(render_fn, gt=(0.60, -0.04, math.pi / 4), step=0.04) -> C1Workload:
    """The C1 scene (render_fn renders the GT object into the table scene) and its 128 candidate poses."""
    from .recognizer import preprocessing_transform
    from .tabletop import yaw_pose_matrix
    names = ["003_cracker_box"]
    bank = syn.model_bank(names)
    pre = preprocessing_transform(bank.models[0], six_dof=False)
    sc = syn.make_tabletop_scene(names, [gt], [pre], render_fn, table_height=0.7,
                                 rng=np.random.default_rng(syn.SEED))
    optical_inv = np.linalg.inv(sc.camera_pose @ syn.CAM_TO_BODY)
    states, mats = [], []
    for ix in range(4):
        for iy in range(4):
            for k in range(8):
                x, y, yaw = gt[0] + (ix - 2) * step, gt[1] + (iy - 2) * step, k * math.pi / 4
                states.append((x, y, yaw))
                mats.append(optical_inv @ yaw_pose_matrix(x, y, sc.table_height, yaw) @ pre)
    gt_index = (2 * 4 + 2) * 8 + 1
    div = np.float32(sc.depth_factor) / np.float32(100.0)
    src_cm = (sc.depth_raw.astype(np.float32) / div).astype(np.int32)
    return C1Workload(sc, init_from_eigen_batch(np.stack(mats)), np.array(states), gt_index, src_cm)
