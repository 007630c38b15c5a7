"""Host orchestration of the GPU greedy-render search: the ObjectRecognizer / EnvObjectRecognition path
that the reference drives through perch_fat (SURVEY.md 8b "secondary seams", build plan step 7).

Mirrors, on top of PoseCore (the C ABI):
  ObjectRecognizer::SetStaticInput / LocalizeObjectsGreedyRender   object_recognizer.cpp:285-342
  EnvObjectRecognition::SetInput (6-DoF images)                     search_env.cpp:5862-6060
  EnvObjectRecognition::ComputeGreedyRenderPoses                    search_env.cpp:2462-2651
  EnvObjectRecognition::GenerateSuccessorStates (pose lists)        search_env.cpp:7056-7254, IsValidPose 309-528
  EnvObjectRecognition::ComputeGreedyCostsInParallelGPU             search_env.cpp:1782-2052
  EnvObjectRecognition::GetStateImagesUnifiedGPU (pose building)    search_env.cpp:1505-1717
and writes perch_fat's output_poses.txt / output_stats.txt (perch_fat.cpp:302-323).

Multi-GPU: with torch.distributed initialised, every rank evaluates a contiguous shard of the candidate
list; the per-model selection keys meet in ONE all-reduce(MIN) and the winning adjusted poses in one
all-reduce(SUM) of a num_models x 16 tensor that only the owning ranks fill.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Union

import numpy as np
import torch

from . import io as pio
from ._native import COST_DEPTH_6DOF, ICP_K, ICP_MAX_ITER, ICP_ROT_EPS, ICP_TRANS_EPS, PCORE_KEY_NONE
from .core import PoseCore, decode_keys
from .distributed import allreduce_min_keys, shard_range
from .model import (Model, chain_matmul_batch, compute_proj, init_from_eigen_batch, matmul_lazy, pose_matrix_batch,
                    quat_from_matrix_eigen_batch, so3_log_batch)

# cam_to_body (search_env.cpp:1536-1539)
CAM_TO_BODY = np.array([[0, 0, 1, 0], [-1, 0, 0, 0], [0, -1, 0, 0], [0, 0, 0, 1]], np.float64)
K_MESH_ADDITIVE_INFLATION = 0.01  # object_model.cpp:43


@dataclass
class PerchParams:
    """perch_params of sbpl_perception/config/pr3_env_config.yaml (6-DoF GPU settings) + defaults of
    search_env.cpp:153-188."""
    icp_type: int = 3                        # 3 = GICP inside the GPU flow
    sensor_resolution: float = 0.01          # sensor_resolution_radius (m)
    min_neighbor_points_for_valid_pose: int = 30
    gpu_batch_size: int = 700
    gpu_stride: int = 8
    gpu_occlusion_threshold: float = 1.0     # cm (search_env.cpp:185)
    gpu_depth_factor: int = 100              # search_env.h:411
    use_color_cost: bool = False
    color_distance_threshold: float = 15.0
    use_cylinder_observed: bool = False      # 3-DoF observed totals from the pose's cylinder
    # IsValidPose's grid-cell radius (search_env.cpp:336-349): env_params_.res = /search_resolution_translation
    # (object_recognizer.cpp:59-60, default 0.04 m), or the model's own with use_model_specific_search_resolution
    search_resolution: float = 0.04
    use_model_specific_search_resolution: bool = False
    depth_median_blur: int = 17              # 3-DoF 8-bit depth: medianBlur aperture (search_env.cpp:187, 5922)
    # fast_gicp settings hard-coded at renderer.cu:1696-1699
    icp_k: int = ICP_K
    icp_max_iterations: int = ICP_MAX_ITER
    icp_rotation_epsilon: float = ICP_ROT_EPS
    icp_transformation_epsilon: float = ICP_TRANS_EPS


@dataclass
class CameraIntrinsics:
    width: int
    height: int
    fx: float
    fy: float
    cx: float
    cy: float


@dataclass
class ModelMetaData:
    """utils.h:82-103 (name, file, flipped, symmetric, ...); `model` may be given instead of `file`."""
    name: str
    file: Optional[str] = None
    model: Optional[Model] = None
    flipped: bool = False
    symmetric: bool = False
    symmetry_mode: int = 0                   # 1 = semi-symmetric (yaw grid stops past pi)
    mesh_in_mm: bool = False
    mesh_scaling_factor: float = 1.0
    search_resolution: float = 0.04          # used with use_model_specific_search_resolution


@dataclass
class RecognitionInput:
    """utils.h:43-80, the fields the 6-DoF GPU path reads."""
    model_names: List[str]
    input_depth_image: Union[str, np.ndarray]          # 16-bit depth (path or (H,W) array)
    predicted_mask_image: Union[str, np.ndarray]       # labels 1..K in model_names order, 0 = background
    depth_factor: float = 10000.0
    camera_pose: np.ndarray = field(default_factory=lambda: np.linalg.inv(CAM_TO_BODY))
    rendered_root_dir: Optional[str] = None             # <root>/<model>/poses.txt
    pose_lists: Optional[Dict[str, np.ndarray]] = None  # alternative: name -> (N, 7) x y z qx qy qz qw
    use_external_pose_list: int = 1
    use_icp: int = 1


@dataclass
class EnvStats:
    """utils.h:114-120."""
    scenes_rendered: int = 0
    scenes_valid: int = 0
    time: float = 0.0
    icp_time: float = 0.0
    peak_gpu_mem: float = 0.0


class States:
    """The candidate states of one search as arrays (the reference's vector<GraphState>): model id, required object
    id (the pose's segmentation label; -1 in 3-DoF) and the pose row -- (x y z qx qy qz qw) for 6-DoF pose lists,
    (x y z yaw) for the 3-DoF grid.  Iterating (or indexing with an int) yields (model, required, pose) tuples; a
    slice is a States."""

    def __init__(self, model=None, req=None, pose=None, width: int = 7):
        self.model = np.zeros(0, np.int32) if model is None else np.ascontiguousarray(model, np.int32)
        self.req = np.zeros(0, np.int32) if req is None else np.ascontiguousarray(req, np.int32)
        self.pose = (np.zeros((0, width), np.float64) if pose is None
                     else np.ascontiguousarray(pose, np.float64).reshape(len(self.model), -1))

    @staticmethod
    def concat(parts: Sequence["States"], width: int = 7) -> "States":
        parts = [p for p in parts if len(p)]
        if not parts:
            return States(width=width)
        return States(np.concatenate([p.model for p in parts]), np.concatenate([p.req for p in parts]),
                      np.concatenate([p.pose for p in parts]))

    def __len__(self):
        return len(self.model)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return States(self.model[i], self.req[i], self.pose[i])
        return int(self.model[i]), int(self.req[i]), self.pose[i]

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]


@dataclass
class LocalizationResult:
    object_transforms: List[np.ndarray]
    preprocessing_transforms: List[np.ndarray]
    detected_poses: List[np.ndarray]     # (7,) x y z qx qy qz qw (ContPose)
    model_names: List[str]
    costs: List[int]
    indices: List[int]
    stats: EnvStats


def preprocessing_transform(model: Model, flipped: bool = False, mesh_in_mm: bool = False,
                            scale: float = 1.0, six_dof: bool = True) -> np.ndarray:
    """PreprocessModel (object_model.cpp:49-132): translate by -centroid (z: centroid for 6-DoF, min z
    otherwise) of the mesh vertices, optional scale and z flip; returns the 4x4 (float32 precision)."""
    v = model.vertices().astype(np.float64)
    c = v.mean(0) if len(v) else np.zeros(3)
    flip = np.eye(4)
    if flipped:
        flip[2, 2] = -1
        v = v * np.array([1, 1, -1])
    z = c[2] if six_dof else (v[:, 2].min() if len(v) else 0.0)
    s = scale if mesh_in_mm else 1.0
    T = np.eye(4)
    T[:3, :3] *= s
    T[:3, 3] = -np.array([c[0] * s, c[1] * s, z * s])
    return (T @ flip).astype(np.float32).astype(np.float64)


def radius_counts(queries: np.ndarray, points: np.ndarray, radius: float, device, cap: Optional[int] = None
                  ) -> np.ndarray:
    """Neighbour counts of PCL's KdTreeFLANN radiusSearch (pcl::search::KdTree over FLANN's exact single-index
    tree), as IsValidPose (search_env.cpp:359-396) and the cylinder totals (search_env.cpp:1593-1612) call it: query
    and points are float PointXYZ, the radius is passed squared as float(r * r), FLANN's L2_Simple sums (q - p)^2 over
    x, y, z in float from zero, and RadiusResultSet keeps a point when dist < r^2 (strict); max_nn (`cap`) caps the
    count.  Elementwise float32 tensor ops on `device`, chunked: each is one IEEE operation, so the counts do not
    depend on the device."""
    q = np.ascontiguousarray(np.asarray(queries, np.float64).astype(np.float32)).reshape(-1, 3)
    pts = np.ascontiguousarray(np.asarray(points, np.float32)).reshape(-1, 3)
    out = np.zeros(len(q), np.int64)
    if len(pts) == 0 or len(q) == 0:
        return out
    r2 = torch.tensor(np.float32(radius * radius), device=device)
    sg = torch.from_numpy(pts).to(device)
    tt = torch.from_numpy(q).to(device)
    step = max(1, (1 << 24) // max(len(pts), 1))
    for a in range(0, len(q), step):
        t = tt[a:a + step]
        dx = t[:, 0:1] - sg[None, :, 0]
        d2 = dx * dx
        dy = t[:, 1:2] - sg[None, :, 1]
        d2 = d2 + dy * dy
        dz = t[:, 2:3] - sg[None, :, 2]
        d2 = d2 + dz * dz
        out[a:a + step] = (d2 < r2).sum(1).cpu().numpy()
    if cap is not None:
        out = np.minimum(out, cap)
    return out


def valid_pose_mask(translations: np.ndarray, seg_points: np.ndarray, search_rad: float, need: int,
                    device) -> np.ndarray:
    """IsValidPose's neighbour test (search_env.cpp:359-396): the pose translation as a float PointXYZ
    (search_env.cpp:317-325) has at least `need` points within search_rad (radius_counts; max_nn = need only caps
    the count)."""
    seg = np.asarray(seg_points, np.float32).reshape(-1, 3)
    if len(seg) < need:
        return np.zeros(len(np.asarray(translations).reshape(-1, 3)), bool)
    return radius_counts(translations, seg, search_rad, device) >= need


def cvtt_i32(x) -> np.ndarray:
    """C++ (int) of floats on x86 (cvttss2si): truncation toward zero; NaN and out-of-range values give INT_MIN."""
    x = np.asarray(x, np.float32)
    with np.errstate(invalid="ignore"):
        ok = np.isfinite(x) & (x > -2147483649.0) & (x < 2147483648.0)
        return np.where(ok, np.trunc(np.where(ok, x, 0.0)), -2147483648).astype(np.int64)


def _dims(model: Model):
    """Bounding-box extents of the model's vertices (min / max over the triangle corners: the same as over
    the unique vertices, without sorting them)."""
    v = model.tris.reshape(-1, 3)
    if len(v) == 0:
        return np.zeros(3)
    return v.max(0).astype(np.float64) - v.min(0).astype(np.float64)


class ObjectRecognizer:
    """ObjectRecognizer + EnvObjectRecognition for the greedy GPU search, driven by PoseCore."""

    # 6-DoF: the successor states stay on the device between IsValidPose and the search launch (TabletopRecognizer
    # builds its 3-DoF states and inputs on the host)
    _device_state_path = True

    def __init__(self, model_bank: Dict[str, ModelMetaData], camera: CameraIntrinsics,
                 params: Optional[PerchParams] = None, device: int = 0):
        self.bank = model_bank
        self.cam = camera
        self.params = params or PerchParams()
        self.device = torch.device("cuda", device)
        self.core = PoseCore(device)
        self.proj = compute_proj(camera.fx, camera.fy, camera.cx, camera.cy, camera.width, camera.height)
        self.core.set_camera(camera.width, camera.height, camera.fx, camera.fy, camera.cx, camera.cy, self.proj)
        self.models: List[Model] = []
        self.model_names: List[str] = []
        self.preprocess: List[np.ndarray] = []
        self.last_stats = EnvStats()
        self.last_timing: dict = {}
        # EnvObjectRecognition::debug_dir_: when set, compute_greedy_render_poses writes <debug_dir>/cost_dump.json
        # (search_env.cpp:2463-2464, 2600-2619, 2647-2649); perch_fat sets it to the experiment directory
        self.debug_dir: Optional[str] = None

    # -- ObjectRecognizer::SetStaticInput -> LoadObjFiles (search_env.cpp:253-307) -----------------
    def set_static_input(self, model_names: Sequence[str], six_dof: bool = True):
        self.models, self.preprocess, self.model_names = [], [], list(model_names)
        self._pre_dev = None  # device copy of the preprocessing transforms (_poses_device)
        for name in model_names:
            meta = self.bank[name]
            m = meta.model if meta.model is not None else pio.load_ply(meta.file, name)
            self.models.append(m)
            self.preprocess.append(preprocessing_transform(m, meta.flipped, meta.mesh_in_mm,
                                                           meta.mesh_scaling_factor, six_dof))
        tris = np.concatenate([m.tris for m in self.models])
        colors = np.concatenate([m.colors for m in self.models])
        self.core.upload_meshes(tris, [m.num_tris for m in self.models], colors)

    # -- SetInput (search_env.cpp:5862-6060), 6-DoF images ------------------------------------------
    def set_input(self, inp: RecognitionInput):
        depth = inp.input_depth_image
        depth = pio.load_depth_png(depth) if isinstance(depth, str) else np.asarray(depth, np.int32)
        mask = inp.predicted_mask_image
        mask = pio.load_mask_png(mask) if isinstance(mask, str) else np.asarray(mask, np.uint8)
        if depth.shape != (self.cam.height, self.cam.width) or mask.shape != depth.shape:
            raise ValueError("depth / mask size does not match the camera")
        p = self.params
        self.camera_pose = np.asarray(inp.camera_pose, np.float64)
        d_depth = torch.from_numpy(np.ascontiguousarray(depth, np.int32)).to(self.device)
        d_mask = torch.from_numpy(np.ascontiguousarray(mask)).to(self.device)
        # depth2cloud_global with the label mask (search_env.cpp:5993-6017)
        self.obs_xyz, self.obs_label = self.core.observed_cloud(d_depth, d_mask, p.gpu_stride, inp.depth_factor)
        lab = self.obs_label.cpu().numpy()
        self.obs_xyz_host = self.obs_xyz.cpu().numpy()
        self.obs_label_host = lab
        K = len(inp.model_names)
        # segmented_observed_point_count (search_env.cpp:6024-6059)
        self.segmented_count = np.bincount(lab[lab >= 0], minlength=K).astype(np.float32)[:max(K, 1)]
        # source depth in gpu cm units: int32 /= (depth_factor / gpu_depth_factor) (search_env.cpp:2487-2498)
        div = np.float32(inp.depth_factor) / np.float32(p.gpu_depth_factor)
        src_cm = (depth.astype(np.float32) / div).astype(np.int32)
        self.core.set_observation(torch.from_numpy(src_cm).to(self.device), d_mask, self.obs_xyz, self.obs_label,
                                  p.sensor_resolution)
        self.segmented_object_names = list(inp.model_names)

    # -- GenerateSuccessorStates (search_env.cpp:7056-7254) ----------------------------------------
    def _model_dims(self, model_id: int) -> np.ndarray:
        """_dims of a model, computed once per model list (the min / max over every triangle corner is the
        slowest part of a search's state generation otherwise)."""
        memo = getattr(self, "_dims_memo", None)
        if memo is None or memo[0] is not self.models:
            memo = self._dims_memo = (self.models, {})
        if model_id not in memo[1]:
            memo[1][model_id] = _dims(self.models[model_id])
        return memo[1][model_id]

    def _search_radius(self, model_id: int) -> float:
        """IsValidPose's search radius, 6-DoF branch (search_env.cpp:336-390): max(inflation * circumscribed
        radius 3D, grid-cell circumscribing radius hypot(res / 2, res / 2)); after_refinement is false on the
        greedy path (search_env.cpp:7140), so the cell term stays."""
        dims = self._model_dims(model_id)
        circ3d = float(max(dims)) / 2.0  # GetCircumscribedRadius3D, object_model.cpp:464-466
        inscribed = float(min(dims[0], dims[1])) / 2.0
        infl = 1.0 + K_MESH_ADDITIVE_INFLATION / inscribed if inscribed > 0 else 1.0  # object_model.cpp:381-383
        p = self.params
        res = p.search_resolution
        if p.use_model_specific_search_resolution:
            res = self.bank[self.model_names[model_id]].search_resolution
        cell = float(np.hypot(res / 2.0, res / 2.0))
        return max(infl * circ3d, cell)

    def _valid_pose_mask(self, model_id: int, translations: np.ndarray, required_object_id: int) -> np.ndarray:
        """IsValidPose (search_env.cpp:309-410), 6-DoF branch: at least min_neighbor_points_for_valid_pose points
        of the object's segmented observed cloud within the search radius, counted as PCL's KdTreeFLANN
        radiusSearch does (valid_pose_mask)."""
        seg = self.obs_xyz_host[self.obs_label_host == required_object_id]
        return valid_pose_mask(translations, seg, self._search_radius(model_id),
                               self.params.min_neighbor_points_for_valid_pose, self.device)

    def _state_lists(self, inp: RecognitionInput):
        """Every model's pose list (poses.txt rows or inp.pose_lists) with its model id, required object id and
        IsValidPose's squared search radius as float32, concatenated in model order; None when there are none."""
        Ps, models, reqs, r2s = [], [], [], []
        for ii, name in enumerate(self.model_names):
            if inp.pose_lists is not None and name in inp.pose_lists:
                P = np.asarray(inp.pose_lists[name], np.float64).reshape(-1, 7)
            elif inp.rendered_root_dir is not None:
                path = os.path.join(inp.rendered_root_dir, name, "poses.txt")
                P = pio.read_poses_txt_cached(path) if os.path.exists(path) else np.zeros((0, 7))
            else:
                P = np.zeros((0, 7))
            if not len(P):
                continue
            req = self.segmented_object_names.index(name) if name in self.segmented_object_names else \
                len(self.segmented_object_names)
            rad = self._search_radius(ii)
            Ps.append(P)
            models.append(np.full(len(P), ii, np.int32))
            reqs.append(np.full(len(P), req, np.int32))
            r2s.append(np.full(len(P), np.float32(rad * rad), np.float32))
        if not Ps:
            return None
        return np.concatenate(Ps), np.concatenate(models), np.concatenate(reqs), np.concatenate(r2s)

    def generate_successor_states(self, inp: RecognitionInput) -> States:
        """GenerateSuccessorStates (search_env.cpp:7056-7254) over every model's pose list, IsValidPose for all of
        them in one device call (pcore_count_within: PCL radiusSearch counts in the required object's segment)."""
        t0 = time.perf_counter()
        lists = self._state_lists(inp)
        if lists is None:
            return States()
        P, model, req, r2 = lists
        t1 = time.perf_counter()
        dev = self.device
        q = torch.from_numpy(np.ascontiguousarray(P[:, :3])).to(dev).float()  # float PointXYZ of the translation
        counts = self.core.count_within(q, torch.from_numpy(req).to(dev), torch.from_numpy(r2).to(dev)).cpu().numpy()
        t2 = time.perf_counter()
        ok = counts >= self.params.min_neighbor_points_for_valid_pose
        out = States(model[ok], req[ok], P[ok])
        self.states_timing = {"lists_s": t1 - t0, "valid_s": t2 - t1, "filter_s": time.perf_counter() - t2}
        return out

    def _successor_states_device(self, inp: RecognitionInput):
        """generate_successor_states with the states kept on the device: (model int32, required object int32, pose
        float64 x 7) tensors of the states that pass IsValidPose, in the same order, or None.  The pose rows go to
        the device once; the filter is a device index (the 6-DoF search path)."""
        t0 = time.perf_counter()
        lists = self._state_lists(inp)
        if lists is None:
            return None
        P, model, req, r2 = lists
        t1 = time.perf_counter()
        dev = self.device
        P_d = torch.from_numpy(P).to(dev)
        req_d = torch.from_numpy(req).to(dev)
        counts = self.core.count_within(P_d[:, :3].float(), req_d, torch.from_numpy(r2).to(dev))
        keep = torch.nonzero(counts >= self.params.min_neighbor_points_for_valid_pose).squeeze(1)
        t2 = time.perf_counter()
        out = (torch.from_numpy(model).to(dev)[keep], req_d[keep], P_d[keep])
        self.states_timing = {"lists_s": t1 - t0, "valid_s": t2 - t1, "filter_s": time.perf_counter() - t2}
        return out

    # -- per-state inputs of the GPU call (GetStateImagesUnifiedGPU, search_env.cpp:1577-1620) -------
    def _cost_type(self) -> int:
        return COST_DEPTH_6DOF

    def _pose_labels(self, states: States) -> Optional[torch.Tensor]:
        """pose_segmentation_label: the state's required object id (6-DoF)."""
        return torch.from_numpy(states.req.copy()).to(self.device)

    def _obs_totals(self, states: States) -> np.ndarray:
        """pose_observed_points_total: segmented_observed_point_count of the label (6-DoF)."""
        seg = np.append(self.segmented_count, 0.0).astype(np.float32)
        return seg[np.minimum(states.req, len(seg) - 1)]

    # the same two inputs on the device path (_device_state_path): device tensors of the states' required object ids
    # in, device tensors out.  A subclass that overrides a host hook overrides its device twin too, or turns the
    # device path off (_check_state_hooks refuses the mix, which would silently use the 6-DoF inputs).
    def _pose_labels_dev(self, req: torch.Tensor) -> Optional[torch.Tensor]:
        """_pose_labels on the device: the required object id (6-DoF)."""
        return req.contiguous()

    def _obs_totals_dev(self, req: torch.Tensor) -> torch.Tensor:
        """_obs_totals on the device: segmented_observed_point_count[req], 0 past the segmented objects."""
        seg = torch.from_numpy(np.append(self.segmented_count, 0.0).astype(np.float32)).to(req.device)
        return seg[torch.clamp(req, max=seg.shape[0] - 1).long()]

    def _check_state_hooks(self):
        if not self._device_state_path:
            return
        cls = type(self)
        for host, dev in (("_pose_labels", "_pose_labels_dev"), ("_obs_totals", "_obs_totals_dev")):
            if getattr(cls, host) is not getattr(ObjectRecognizer, host) and \
                    getattr(cls, dev) is getattr(ObjectRecognizer, dev):
                raise TypeError(f"{cls.__name__} overrides {host} but not {dev}: override both, or set "
                                f"_device_state_path = False")

    def _poses_device(self, states) -> torch.Tensor:
        """The states' search poses on the device (pcore_state_poses: _pose_in_cam's arithmetic, bit for bit)."""
        if not len(states):
            return torch.zeros((0, 16), dtype=torch.float32, device=self.device)
        st = torch.from_numpy(np.ascontiguousarray(states.pose, np.float64)).to(self.device)
        return self._state_poses_dev(st, torch.from_numpy(states.model.copy()).to(self.device))

    def _state_poses_dev(self, pose: torch.Tensor, model: torch.Tensor) -> torch.Tensor:
        """pcore_state_poses of device state rows (float64 x 7) and model ids."""
        cam_matrix = np.linalg.inv(self.camera_pose @ CAM_TO_BODY)
        if getattr(self, "_pre_dev", None) is None or self._pre_dev.shape[0] != len(self.preprocess):
            self._pre_dev = torch.from_numpy(np.stack(self.preprocess).reshape(-1, 16).astype(np.float64)).to(self.device)
        return self.core.state_poses(pose.contiguous(), model.contiguous(), cam_matrix, self._pre_dev)

    def _pose_in_cam(self, states) -> np.ndarray:
        """GetStateImagesUnifiedGPU pose building (search_env.cpp:1535-1576) on the host: inv(cam_z_front) *
        T(state) * preprocess, vectorised over the states (model.chain_matmul_batch: index-order 4x4 products);
        the restatement pcore_state_poses is held to."""
        cam_z_front = self.camera_pose @ CAM_TO_BODY
        cam_matrix = np.linalg.inv(cam_z_front)
        if not len(states):
            return init_from_eigen_batch(np.zeros((0, 4, 4)), 100)
        P = states.pose
        pre = np.stack(self.preprocess)[states.model]
        mats = chain_matmul_batch(cam_matrix, pose_matrix_batch(P[:, :3], P[:, 3:7]), pre)
        return init_from_eigen_batch(mats, 100)

    # -- ComputeGreedyRenderPoses (search_env.cpp:2462-2651) ----------------------------------------
    def compute_greedy_render_poses(self, inp: RecognitionInput):
        t0 = time.perf_counter()
        p = self.params
        self._check_state_hooks()
        if self._device_state_path:
            dstates = self._successor_states_device(inp)
            n_total = 0 if dstates is None else int(dstates[0].shape[0])
        else:
            states = self.generate_successor_states(inp)
            n_total = len(states)
        t_states = time.perf_counter()
        K = len(self.models)
        world, rank = 1, 0
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            world, rank = torch.distributed.get_world_size(), torch.distributed.get_rank()
        lo, hi = shard_range(n_total, rank, world)
        n = hi - lo
        keys = torch.full((K,), PCORE_KEY_NONE, dtype=torch.int64, device=self.device)
        adj_all = None
        icp_time = 0.0
        gpu_s = 0.0
        peak_mb = float(torch.cuda.max_memory_allocated(self.device)) / 1024.0 / 1024.0
        t_build = t_states
        if n > 0:
            if self._device_state_path:
                model_d, req_d, pose_d = (t[lo:hi] for t in dstates)
                poses = self._state_poses_dev(pose_d, model_d)
                pm = model_d.contiguous()
                pl = self._pose_labels_dev(req_d)  # pose_segmentation_label
                tot = self._obs_totals_dev(req_d)  # pose_observed_points_total
            else:
                mine = states[lo:hi]
                poses = self._poses_device(mine)
                pm = torch.from_numpy(mine.model.copy()).to(self.device)
                pl = self._pose_labels(mine)
                tot = torch.from_numpy(self._obs_totals(mine)).to(self.device)
            cost_type = self._cost_type()
            rc = torch.empty(n, dtype=torch.float32, device=self.device)
            oc = torch.empty_like(rc)
            df = torch.empty_like(rc)
            adj_all = poses.clone()
            iters = torch.zeros(n, dtype=torch.int32, device=self.device)
            t_build = time.perf_counter()
            # The reference loops over gpu_batch_size batches (search_env.cpp:2504-2525) only to bound its
            # per-call device allocations; the results are batch-invariant (the keys fold across batches, tests/
            # test_gpu_fullsize.py::test_c2_permutation_and_chunking_invariance) and the context chunks GICP by
            # its own scratch budget, so the whole shard goes down in one call.
            ti = time.perf_counter()
            if p.icp_type == 3 and inp.use_icp:
                self.core.evaluate_icp(poses, pm, pl, tot, cost_type=cost_type, stride=p.gpu_stride,
                                       depth_factor=p.gpu_depth_factor, sensor_resolution=p.sensor_resolution,
                                       occlusion_threshold=p.gpu_occlusion_threshold, k=p.icp_k,
                                       max_iterations=p.icp_max_iterations, rotation_epsilon=p.icp_rotation_epsilon,
                                       transformation_epsilon=p.icp_transformation_epsilon,
                                       out=(adj_all, iters, rc, oc, df))
                self.core.select(rc, oc, pm, K, index_base=lo, keys=keys)
            else:  # the argmin keys folded in the scoring launch (pcore_evaluate_select)
                self.core.evaluate(poses, pm, pl, tot, cost_type=cost_type, stride=p.gpu_stride,
                                   depth_factor=p.gpu_depth_factor, sensor_resolution=p.sensor_resolution,
                                   occlusion_threshold=p.gpu_occlusion_threshold, out=(rc, oc, df),
                                   select=(keys, lo, K))
            torch.cuda.synchronize(self.device)
            gpu_s = time.perf_counter() - ti
            if p.icp_type == 3 and inp.use_icp:
                # gpu_stats of the call (renderer.cu:1736-1739): the GICP stage's own time and the peak memory;
                # search_env.cpp:1715-1716 adds icp_runtime (seconds) to env_stats_.icp_time
                st = self.core.stats(reset=True)
                icp_time = float(st["icp_runtime"])
                peak_mb = st["peak_memory_usage"]  # gpu_stats.peak_memory_usage (MB)
            self._last_costs_dev = (rc, oc, df)  # read back only on request (_last_costs)
        allreduce_min_keys(keys)
        cost, idx = decode_keys(keys)
        # winning adjusted poses: the owning rank contributes, the others add zeros
        win = torch.zeros((K, 16), dtype=torch.float32, device=self.device)
        for m in range(K):
            if idx[m] >= 0 and lo <= idx[m] < hi:
                win[m] = adj_all[int(idx[m]) - lo]
        if world > 1:
            torch.distributed.all_reduce(win, op=torch.distributed.ReduceOp.SUM)
            # stats: the slowest rank's GICP stage and the largest peak memory (the shards run concurrently)
            st = torch.tensor([icp_time, peak_mb], dtype=torch.float64, device=self.device)
            torch.distributed.all_reduce(st, op=torch.distributed.ReduceOp.MAX)
            icp_time, peak_mb = float(st[0]), float(st[1])
        win = win.cpu().numpy()
        found = [m for m in range(K) if idx[m] >= 0]
        conts = self.adjusted_cont_poses(win[found], np.array(found, np.int32), inp.use_external_pose_list)
        results = [(m, int(cost[m]), int(idx[m]), conts[r]) for r, m in enumerate(found)]
        dump = self.debug_dir is not None
        if world > 1:  # rank 0's debug_dir decides, so every rank takes part in the gather
            flag = torch.tensor([1 if dump else 0], dtype=torch.int32, device=self.device)
            torch.distributed.broadcast(flag, src=0)
            dump = bool(flag.item())
        if dump:
            self._write_cost_dump(inp, n_total, lo, n, adj_all if n > 0 else None, pm if n > 0 else None, world, rank)
        t_end = time.perf_counter()
        # host-side breakdown of the last search (seconds): successor states (poses.txt + IsValidPose), per-state
        # inputs of the GPU call, the GPU search (launch .. synchronise, incl. the exchange), results
        self.last_timing = {"states_s": t_states - t0, "inputs_s": t_build - t_states,
                            "gpu_s": gpu_s, "total_s": t_end - t0, **getattr(self, "states_timing", {})}
        self.last_stats = EnvStats(scenes_rendered=n_total, scenes_valid=0, time=time.perf_counter() - t0,
                                   icp_time=icp_time, peak_gpu_mem=peak_mb)
        return results

    def adjusted_cont_poses(self, adj16: np.ndarray, model: np.ndarray, use_external_pose_list: int) -> np.ndarray:
        """ComputeGreedyCostsInParallelGPU's adjusted ContPose of each state (search_env.cpp:1996-2019): the GPU-adjusted
        mat4x4 -> to_eigen(100) (a Matrix4f); in 3-DoF cam_z_front * T * preprocess^-1 as float products; then
        (T(0,3), T(1,3), T(2,3)) and Quaternionf of the float rotation block.  -> (N, 7) x y z qx qy qz qw."""
        A = np.asarray(adj16, np.float32).reshape(-1, 4, 4).copy()
        A[:, :3, :] = A[:, :3, :] / np.float32(100.0)
        if use_external_pose_list != 1 and len(A):
            cz = (self.camera_pose @ CAM_TO_BODY).astype(np.float32)
            pinv = np.stack([np.linalg.inv(P).astype(np.float32) for P in self.preprocess])[np.asarray(model)]
            A = matmul_lazy(matmul_lazy(np.broadcast_to(cz, A.shape), A), pinv)
        q = quat_from_matrix_eigen_batch(A[:, :3, :3], np.float32)
        return np.concatenate([A[:, :3, 3], q], 1).astype(np.float64)

    def raw_model_to_scene(self, cont: np.ndarray, model: np.ndarray) -> np.ndarray:
        """ObjectModel::GetRawModelToSceneTransform (object_model.cpp:502-510) of ContPoses (N, 7): GetTransform() (double:
        translation * normalised quaternion) cast to float, times the float preprocessing transform.  -> (N, 4, 4)
        float32."""
        c = np.asarray(cont, np.float64).reshape(-1, 7)
        if not len(c):
            return np.zeros((0, 4, 4), np.float32)
        T = pose_matrix_batch(c[:, :3], c[:, 3:7]).astype(np.float32)
        pre = np.stack([P.astype(np.float32) for P in self.preprocess])[np.asarray(model)]
        return matmul_lazy(T, pre)

    def _write_cost_dump(self, inp, n_total, lo, n, adj, pm, world, rank):
        """<debug_dir>/cost_dump.json as ComputeGreedyRenderPoses writes it (search_env.cpp:2540-2649): one entry per
        candidate state whose cost is not -1 / -2, in candidate order -- id (the state's index), target_cost = (int) rc,
        source_cost = (int) oc, total_cost = (int) (rc + oc), transform (GetRawModelToSceneTransform of the adjusted
        pose, column-major), translation, quaternion (x y z w) and lie_rotation (Sophus SO3f log).  The costs are the
        ones this search's argmin used, read back from the device outputs it already holds (no extra launch); with
        several ranks the kept rows of every shard are gathered on rank 0, which writes the file into its debug_dir
        (every rank calls this when rank 0's debug_dir is set)."""
        if n > 0:
            rc, oc, _ = self._last_costs
            adj_h, pm_h = adj.cpu().numpy(), pm.cpu().numpy()
        else:
            rc = oc = np.zeros(0, np.float32)
            adj_h, pm_h = np.zeros((0, 16), np.float32), np.zeros(0, np.int32)
        target, source = cvtt_i32(rc), cvtt_i32(oc)
        total = cvtt_i32(np.asarray(rc, np.float32) + np.asarray(oc, np.float32))
        cost = np.where(target < 0, -1, total)
        keep = np.nonzero((cost != -1) & (cost != -2))[0]
        ids, target, source, cost = keep + lo, target[keep], source[keep], cost[keep]
        adj_h, pm_h = adj_h[keep], pm_h[keep]
        if world > 1:  # only the kept rows travel
            parts = [None] * world
            torch.distributed.all_gather_object(parts, (lo, ids, target, source, cost, adj_h, pm_h))
            if rank != 0:
                return
            parts.sort(key=lambda p: p[0])
            ids, target, source, cost, adj_h, pm_h = (np.concatenate([p[k] for p in parts]) for k in range(1, 7))
        cont = self.adjusted_cont_poses(adj_h, pm_h, inp.use_external_pose_list)
        T = self.raw_model_to_scene(cont, pm_h)
        lie = so3_log_batch(quat_from_matrix_eigen_batch(T[:, :3, :3], np.float32), np.float32)
        c32 = cont.astype(np.float32)
        poses = []
        for r in range(len(ids)):
            poses.append({"id": int(ids[r]), "target_cost": int(target[r]), "source_cost": int(source[r]),
                          "total_cost": int(cost[r]),
                          "transform": [float(v) for v in T[r].T.reshape(-1)],  # Eigen's column-major data()
                          "translation": [float(v) for v in c32[r, :3]],
                          "quaternion": [float(v) for v in c32[r, 3:7]],
                          "lie_rotation": [float(v) for v in lie[r]]})
        pio.write_cost_dump(os.path.join(self.debug_dir, "cost_dump.json"), poses)

    @property
    def _last_costs(self):
        """The last search's per-state rendered / observed / points-diff costs as numpy arrays (diagnostics)."""
        return tuple(t.cpu().numpy() for t in self._last_costs_dev)

    # -- ObjectRecognizer::LocalizeObjectsGreedyRender (object_recognizer.cpp:290-342) -------------
    def localize_objects_greedy_render(self, inp: RecognitionInput) -> LocalizationResult:
        if not self.models or self.model_names != list(inp.model_names):
            self.set_static_input(inp.model_names, six_dof=inp.use_external_pose_list == 1)
        t0 = time.perf_counter()
        self.set_input(inp)
        t_input = time.perf_counter() - t0
        res = self.compute_greedy_render_poses(inp)
        self.last_timing["set_input_s"] = t_input
        return self.localization_result(res)

    def localization_result(self, res) -> LocalizationResult:
        """compute_greedy_render_poses' (model, cost, index, ContPose) tuples -> the outputs of
        LocalizeObjectsGreedyRender (object_recognizer.cpp:318-337): per detected object the raw-model-to-scene
        transform, the preprocessing transform, the pose and the model name."""
        out = LocalizationResult([], [], [], [], [], [], self.last_stats)
        raw = self.raw_model_to_scene(np.array([r[3] for r in res]).reshape(-1, 7), np.array([r[0] for r in res], np.int32))
        for (m, cost, idx, cont), T in zip(res, raw):
            # GetRawModelToSceneTransform (object_model.cpp:502-510): ContPose transform * preprocessing
            out.object_transforms.append(T.astype(np.float64))
            out.preprocessing_transforms.append(self.preprocess[m])
            out.detected_poses.append(cont)
            out.model_names.append(self.model_names[m])
            out.costs.append(cost)
            out.indices.append(idx)
        return out

    def write_outputs(self, result: LocalizationResult, out_dir: str):
        """perch_fat.cpp:302-323 output_poses.txt + output_stats.txt."""
        os.makedirs(out_dir, exist_ok=True)
        objs = [pio.DetectedObject(n, c[:3], c[3:7], T, P) for n, c, T, P in
                zip(result.model_names, result.detected_poses, result.object_transforms,
                    result.preprocessing_transforms)]
        pio.write_output_poses(os.path.join(out_dir, "output_poses.txt"), objs)
        s = result.stats
        # object_recognizer.cpp:312-318: the planning stats of the greedy search are expands = scenes_rendered,
        # time = the env's time, cost 0
        pio.write_output_stats(os.path.join(out_dir, "output_stats.txt"), s.scenes_rendered, s.scenes_valid,
                               s.scenes_rendered, s.time, 0, s.icp_time, s.peak_gpu_mem)
