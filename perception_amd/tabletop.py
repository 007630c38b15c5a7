"""3-DoF table-top search: the C1-style scenes of the reference's PR2 GPU setup.

Objects stand upright on a table of known height; a candidate is (x, y, yaw) on a grid over the table
region.  Mirrors, on top of PoseCore:

  SetInput, 3-DoF GPU images                 search_env.cpp:5908-5944 (world bounds x_max..z_min with
                                              z in [table, table + 0.5], camera transform cam_to_world
                                              * cam_to_body), 5976-6017 (depth2cloud_global)
  projected cloud for IsValidPose            search_env.cpp:5636-5662 (observed points at z = table)
  GenerateSuccessorStates, 3-DoF grid        search_env.cpp:7268-7320 (x, y from min to max in steps of
                                              res, yaw from 0 in steps of theta_res, IsValidPose, the
                                              semi-symmetric cut)
  IsValidPose, projected branch              search_env.cpp:309-375 (>= min_neighbor_points_for_valid_pose
                                              projected points within max(circumscribed radius, cell
                                              circumradius) of (x, y, table))
  pose_observed_points_total, cylinder       search_env.cpp:1591-1619 (projected points within inflation *
                                              circumscribed radius)
  ContPose(x, y, z, roll, pitch, yaw)        object_state.cpp:17-22, 83-97 (normalize_angle_positive,
                                              yaw * pitch * roll quaternion)

Scoring is the GPU hot path with cost_type 0 (depth) -- or 1 (colour gate) once the observation has
colours -- and no pose labels.  Differences from the reference: the projected cloud is the stride-1
bounded GPU cloud moved to the world frame (the reference builds it on the CPU with PCL from the same
depth image, GetGravityAlignedPointCloud, search_env.cpp:4475-4600, without downsampling by default); the
8-bit depth images (the reference's non-16-bit branch, search_env.cpp:5916-5929) are median-blurred first
(median_blur_u8, OpenCV medianBlur semantics).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ._native import COST_DEPTH_3DOF, COST_RGBD_3DOF
from .model import pose_matrix
from .recognizer import (CAM_TO_BODY, K_MESH_ADDITIVE_INFLATION, CameraIntrinsics, ModelMetaData,
                         ObjectRecognizer, PerchParams, RecognitionInput, States, _dims, radius_counts)


@dataclass
class TableParams:
    """env_params_ of the 3-DoF search (env_config.yaml: search_resolution_translation 0.04 m,
    search_resolution_yaw 0.3926991 rad; table and region bounds come with the input)."""
    x_min: float
    x_max: float
    y_min: float
    y_max: float
    table_height: float
    res: float = 0.04
    theta_res: float = 0.3926991


def pr2_gpu_params(**kw) -> PerchParams:
    """perch_params of config/pr2_gpu_env_config.yaml (3-DoF GPU): stride 4, 7.5 mm sensor radius, 30
    neighbours for a valid pose, colour cost with threshold 11.5, cylinder observed totals, no ICP."""
    p = PerchParams(icp_type=0, sensor_resolution=0.0075, min_neighbor_points_for_valid_pose=30, gpu_stride=4,
                    use_color_cost=True, color_distance_threshold=11.5, use_cylinder_observed=True)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def median_blur_u8(img: np.ndarray, ksize: int, device="cpu") -> np.ndarray:
    """cv::medianBlur of an 8-bit image (search_env.cpp:5922, applied to 8-bit depth before the GPU path): each
    pixel becomes the median of its ksize x ksize window, the border replicated (OpenCV's BORDER_REPLICATE); ksize
    odd and > 1 (ksize 1 copies).  Exact: the window holds an odd number of integers.  Torch ops on `device`
    (unfold + kthvalue), once per scene."""
    a = np.ascontiguousarray(img, np.uint8)
    k = int(ksize)
    if k <= 1:
        return a.copy()
    if k % 2 == 0:
        raise ValueError("medianBlur: ksize must be odd")
    r = k // 2
    t = torch.from_numpy(a).to(device).to(torch.int16)[None, None].float()
    t = torch.nn.functional.pad(t, (r, r, r, r), mode="replicate")
    H, W = a.shape
    out = np.empty((H, W), np.uint8)
    rows = max(1, (1 << 24) // (k * k * W))
    for y0 in range(0, H, rows):
        y1 = min(H, y0 + rows)
        win = torch.nn.functional.unfold(t[:, :, y0:y1 + 2 * r, :], kernel_size=k)  # (1, k*k, rows*W)
        med = win[0].kthvalue(k * k // 2 + 1, dim=0).values
        out[y0:y1] = med.reshape(y1 - y0, W).to(torch.uint8).cpu().numpy()
    return out


def normalize_angle_positive(a: float) -> float:
    """angles::normalize_angle_positive: fmod(fmod(a, 2 pi) + 2 pi, 2 pi)."""
    two_pi = 2.0 * math.pi
    return math.fmod(math.fmod(a, two_pi) + two_pi, two_pi)


def yaw_pose_matrix(x: float, y: float, z: float, yaw: float) -> np.ndarray:
    """ContPose(x, y, z, 0, 0, yaw).GetTransform(): quaternion yaw * pitch * roll with zero roll / pitch is
    (cos(yaw / 2), 0, 0, sin(yaw / 2)), normalised, then Translation3d * rotation."""
    yaw = normalize_angle_positive(yaw)
    return pose_matrix([x, y, z], [0.0, 0.0, math.sin(yaw / 2.0), math.cos(yaw / 2.0)])


def circumscribed_radius(dims) -> float:
    """ObjectModel::GetCircumscribedRadius (object_model.cpp:460-462): half the larger footprint side."""
    return float(max(abs(dims[0]), abs(dims[1]))) / 2.0


def inflation_factor(dims) -> float:
    """object_model.cpp:381-383: 1 + kMeshAdditiveInflation / inscribed radius."""
    inscribed = float(min(dims[0], dims[1])) / 2.0
    return 1.0 + K_MESH_ADDITIVE_INFLATION / inscribed if inscribed > 0 else 1.0


def count_within(centres_xy: np.ndarray, pts_xy: np.ndarray, radius: float, table_height: float = 0.0,
                 device="cpu", cap: Optional[int] = None) -> np.ndarray:
    """Projected-cloud radius search counts: every projected point and every query sits at z = table_height
    (search_env.cpp:5643-5649, 317-325), so the PCL float distance is the (x, y) one (radius_counts)."""
    c = np.asarray(centres_xy, np.float64).reshape(-1, 2)
    p = np.asarray(pts_xy, np.float32).reshape(-1, 2)
    zq = np.full((len(c), 1), table_height, np.float64)
    zp = np.full((len(p), 1), np.float32(table_height), np.float32)
    return radius_counts(np.hstack([c, zq]), np.hstack([p, zp]), radius, device, cap)


def grid_states(table: TableParams, model_id: int, dims, projected_xy: np.ndarray, min_neighbors: int,
                symmetry_mode: int = 0, device="cpu") -> List[tuple]:
    """GenerateSuccessorStates' 3-DoF grid (search_env.cpp:7268-7320) for one model: x and y advance by
    repeated addition of res (double), yaw from 0 below 2 pi by theta_res; a pose needs IsValidPose; for a
    semi-symmetric model (symmetry_mode 1) the yaw loop stops at the first valid yaw above pi + theta_res."""
    cell_r = math.hypot(table.res / 2.0, table.res / 2.0)
    rad = max(circumscribed_radius(dims), cell_r)
    xs, x = [], table.x_min
    while x <= table.x_max:
        xs.append(x)
        x += table.res
    ys, y = [], table.y_min
    while y <= table.y_max:
        ys.append(y)
        y += table.res
    thetas, t = [], 0.0
    while t < 2 * math.pi:
        thetas.append(t)
        t += table.theta_res
    states = []
    for x in xs:
        for y in ys:
            ok = count_within(np.array([[x, y]]), projected_xy, rad, table.table_height, device)[0] >= min_neighbors
            for th in thetas:
                if not ok:
                    continue  # IsValidPose does not depend on yaw in the projected branch
                if symmetry_mode == 1 and th > math.pi + table.theta_res:
                    break
                states.append((model_id, -1, np.array([x, y, table.table_height, th])))
    return states


class TabletopRecognizer(ObjectRecognizer):
    """ObjectRecognizer in the 3-DoF GPU mode (use_external_pose_list = 0)."""

    _device_state_path = False  # the 3-DoF grid states and their inputs are built on the host

    def __init__(self, model_bank: Dict[str, ModelMetaData], camera: CameraIntrinsics, table: TableParams,
                 params: Optional[PerchParams] = None, device: int = 0):
        super().__init__(model_bank, camera, params or pr2_gpu_params(), device)
        self.table = table
        self.obs_rgb = None

    # SetInput, 3-DoF branch (search_env.cpp:5908-6017)
    def set_input_3dof(self, depth: np.ndarray, camera_pose: np.ndarray, depth_factor: float,
                       rgb: Optional[np.ndarray] = None):
        p, tb = self.params, self.table
        if np.asarray(depth).dtype == np.uint8:  # 8-bit depth: medianBlur first (search_env.cpp:5916-5929)
            depth = median_blur_u8(depth, p.depth_median_blur, self.device)
        depth = np.ascontiguousarray(depth, np.int32)
        if depth.shape != (self.cam.height, self.cam.width):
            raise ValueError("depth size does not match the camera")
        self.camera_pose = np.asarray(camera_pose, np.float64)
        self.transform = (self.camera_pose @ CAM_TO_BODY).astype(np.float32)
        self.bounds = [tb.x_max, tb.x_min, tb.y_max, tb.y_min, tb.table_height + 0.5, tb.table_height]
        d_depth = torch.from_numpy(depth).to(self.device)
        d_rgb = None if rgb is None else torch.from_numpy(np.ascontiguousarray(rgb, np.uint8)).to(self.device)
        self.obs_xyz, self.obs_rgb = self.core.observed_cloud_bounded(d_depth, p.gpu_stride, depth_factor,
                                                                      self.transform, self.bounds, rgb=d_rgb)
        self.obs_xyz_host = self.obs_xyz.cpu().numpy()
        self.obs_label_host = np.zeros(len(self.obs_xyz_host), np.int32)
        div = np.float32(depth_factor) / np.float32(p.gpu_depth_factor)
        src_cm = (depth.astype(np.float32) / div).astype(np.int32)
        self.core.set_observation(torch.from_numpy(src_cm).to(self.device), None, self.obs_xyz, None,
                                  p.sensor_resolution)
        self.use_colour = bool(p.use_color_cost and rgb is not None and hasattr(self.core, "set_observation_colors"))
        if self.use_colour:
            self.core.set_observation_colors(self.obs_rgb)
        # projected cloud (search_env.cpp:5636-5662): full-resolution bounded points at the table height
        full, _ = self.core.observed_cloud_bounded(d_depth, 1, depth_factor, self.transform, self.bounds)
        # the world frame in float, row by row left to right (pcl::transformPointCloud with an Affine3f)
        f = full.cpu().numpy().astype(np.float32)
        M = self.transform.astype(np.float32)
        self.projected_xy = np.stack([((M[r, 0] * f[:, 0] + M[r, 1] * f[:, 1]) + M[r, 2] * f[:, 2]) + M[r, 3]
                                      for r in range(2)], 1)
        self.segmented_object_names = []

    def generate_successor_states(self, inp: RecognitionInput = None) -> States:
        parts = []
        for ii, name in enumerate(self.model_names):
            dims = _dims(self.models[ii])
            sym = self.bank[name].symmetry_mode
            st = grid_states(self.table, ii, dims, self.projected_xy,
                             self.params.min_neighbor_points_for_valid_pose, sym, self.device)
            if st:
                parts.append(States(np.array([s[0] for s in st], np.int32), np.array([s[1] for s in st], np.int32),
                                    np.stack([s[2] for s in st])))
        return States.concat(parts, width=4)

    def _cost_type(self) -> int:
        return COST_RGBD_3DOF if getattr(self, "use_colour", False) else COST_DEPTH_3DOF

    def _pose_labels(self, states):
        return None

    def _obs_totals(self, states) -> np.ndarray:
        """Cylinder totals (use_cylinder_observed): projected points within inflation * circumscribed radius
        of the pose (search_env.cpp:1591-1612); else all observed points (1613-1617)."""
        if not self.params.use_cylinder_observed:
            return np.full(len(states), float(len(self.obs_xyz_host)), np.float32)
        out = np.empty(len(states), np.float32)
        for mid in np.unique(states.model):
            sel = states.model == mid
            dims = _dims(self.models[mid])
            r = inflation_factor(dims) * circumscribed_radius(dims)
            out[sel] = count_within(states.pose[sel, :2], self.projected_xy, r, self.table.table_height,
                                    self.device, cap=self.cam.width * self.cam.height)  # max_nn = kNumPixels
        return out

    def _poses_device(self, states) -> torch.Tensor:
        return torch.from_numpy(self._pose_in_cam(states)).to(self.device)

    def _pose_in_cam(self, states) -> np.ndarray:
        """The 3-DoF states' poses in the camera, vectorised (yaw quaternions with math.sin / math.cos per
        state, as yaw_pose_matrix; index-order 4x4 products, model.chain_matmul_batch)."""
        from .model import chain_matmul_batch, init_from_eigen_batch, pose_matrix_batch
        cam_matrix = np.linalg.inv(self.camera_pose @ CAM_TO_BODY)
        if not len(states):
            return init_from_eigen_batch(np.zeros((0, 4, 4)), 100)
        xyzy = states.pose
        yaws = [normalize_angle_positive(float(y)) for y in xyzy[:, 3]]
        q = np.array([(0.0, 0.0, math.sin(y / 2.0), math.cos(y / 2.0)) for y in yaws])
        mats = chain_matmul_batch(cam_matrix, pose_matrix_batch(xyzy[:, :3], q), np.stack(self.preprocess)[states.model])
        return init_from_eigen_batch(mats, 100)

    def localize(self, model_names: Sequence[str], depth: np.ndarray, camera_pose: np.ndarray,
                 depth_factor: float, rgb: Optional[np.ndarray] = None):
        """LocalizeObjectsGreedyRender in 3-DoF mode: (model, cost, index, ContPose x y z qx qy qz qw)."""
        if not self.models or self.model_names != list(model_names):
            self.set_static_input(model_names, six_dof=False)
        self.set_input_3dof(depth, camera_pose, depth_factor, rgb)
        inp = RecognitionInput(list(model_names), depth, np.zeros_like(depth, np.uint8), depth_factor=depth_factor,
                               camera_pose=camera_pose, use_external_pose_list=0, use_icp=0)
        return self.compute_greedy_render_poses(inp)
