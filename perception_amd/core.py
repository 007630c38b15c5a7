"""PoseCore: the device-side context of the pose-search core, driven with PyTorch-ROCm tensors.

This is the Python face of include/pcore.h.  Every array argument of the per-batch calls is a CUDA
(HIP) torch tensor; its data_ptr() goes straight into the C ABI, and the work runs on torch's
current stream.  There is no CPU fallback: a missing libpcore.so or a non-GPU tensor raises.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native
from ._native import Camera, EvalParams, IcpParams, PcoreError


def _ptr(t: Optional[torch.Tensor], dtype: torch.dtype, name: str):
    if t is None:
        return None
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{name}: expected a GPU torch tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: tensor must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def _stream(stream: Optional[torch.cuda.Stream]):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class PoseCore:
    """One context per (host thread, device), like the reference's single-threaded caller
    (search_env.cpp:2506-2525)."""

    def __init__(self, device: int = 0):
        self.lib = _native.load()
        self.device = int(device)
        h = ctypes.c_void_p()
        rc = self.lib.pcore_create(self.device, ctypes.byref(h))
        if rc != _native.PCORE_OK:
            raise PcoreError(rc, f"pcore_create(device={device}) failed")
        self._h = h
        self.width = self.height = 0
        self.num_models = 0

    # -- lifetime ---------------------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.pcore_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc != _native.PCORE_OK:
            msg = self.lib.pcore_last_error(self._h)
            raise PcoreError(rc, msg.decode() if msg else "")

    # -- static inputs ----------------------------------------------------------------------------
    def upload_meshes(self, tris: np.ndarray, tris_model_count, colors: Optional[np.ndarray] = None):
        tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
        cnt = np.ascontiguousarray(tris_model_count, dtype=np.int32)
        col = None if colors is None else np.ascontiguousarray(colors, dtype=np.uint8).reshape(-1, 3)
        self._check(self.lib.pcore_upload_meshes(
            self._h, tris.ctypes.data_as(ctypes.c_void_p),
            None if col is None else col.ctypes.data_as(ctypes.c_void_p), tris.shape[0],
            cnt.ctypes.data_as(ctypes.c_void_p), cnt.shape[0]))
        self.num_models = int(cnt.shape[0])

    def set_camera(self, width: int, height: int, fx: float, fy: float, cx: float, cy: float, proj: np.ndarray):
        cam = Camera()
        cam.width, cam.height = int(width), int(height)
        cam.fx, cam.fy, cam.cx, cam.cy = float(fx), float(fy), float(cx), float(cy)
        pj = np.asarray(proj, dtype=np.float32).reshape(16)
        for i in range(16):
            cam.proj[i] = float(pj[i])
        self._check(self.lib.pcore_set_camera(self._h, ctypes.byref(cam)))
        self.width, self.height = int(width), int(height)

    # -- per-scene inputs -------------------------------------------------------------------------
    def observed_cloud(self, depth: torch.Tensor, label_mask: Optional[torch.Tensor], stride: int,
                       depth_factor: float, stream=None) -> Tuple[torch.Tensor, torch.Tensor]:
        """depth2cloud_global (renderer.cu:1936-2069): returns (xyz (P,3) f32, label (P,) i32) on the GPU."""
        h, w = depth.shape[-2:]
        cap = ((w + stride - 1) // stride) * ((h + stride - 1) // stride)
        xyz = torch.empty((max(cap, 1), 3), dtype=torch.float32, device=depth.device)
        lab = torch.empty((max(cap, 1),), dtype=torch.int32, device=depth.device)
        cnt = ctypes.c_int32(0)
        self._check(self.lib.pcore_observed_cloud(
            self._h, _ptr(depth, torch.int32, "depth"), _ptr(label_mask, torch.uint8, "label_mask"), w, h, stride,
            float(depth_factor), _ptr(xyz, torch.float32, "xyz"), _ptr(lab, torch.int32, "label"), cap,
            ctypes.byref(cnt), _stream(stream)))
        n = cnt.value
        return xyz[:n], lab[:n]

    def observed_cloud_bounded(self, depth: torch.Tensor, stride: int, depth_factor: float,
                               cam_to_world: Optional[np.ndarray] = None, bounds: Optional[Sequence[float]] = None,
                               rgb: Optional[torch.Tensor] = None, stream=None
                               ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        """3-DoF depth2cloud_global: camera-frame points of the pixels whose world point (cam_to_world, 4x4)
        lies inside bounds = (x_max, x_min, y_max, y_min, z_max, z_min); with `rgb` (H, W, 3) uint8 also the
        points' colours.  Returns (xyz (P,3) f32, rgb (P,3) u8 or None) on the GPU."""
        h, w = depth.shape[-2:]
        cap = ((w + stride - 1) // stride) * ((h + stride - 1) // stride)
        xyz = torch.empty((max(cap, 1), 3), dtype=torch.float32, device=depth.device)
        out_rgb = torch.empty((max(cap, 1), 3), dtype=torch.uint8, device=depth.device) if rgb is not None else None
        M = None if cam_to_world is None else (ctypes.c_float * 16)(*np.asarray(cam_to_world, np.float32).reshape(16))
        B = None if bounds is None else (ctypes.c_double * 6)(*np.asarray(bounds, np.float64).reshape(6))
        cnt = ctypes.c_int32(0)
        self._check(self.lib.pcore_observed_cloud_bounded(
            self._h, _ptr(depth, torch.int32, "depth"), _ptr(None if rgb is None else rgb.contiguous(), torch.uint8, "rgb"),
            w, h, stride, float(depth_factor), M, B, _ptr(xyz, torch.float32, "xyz"),
            _ptr(out_rgb, torch.uint8, "out_rgb"), cap, ctypes.byref(cnt), _stream(stream)))
        n = cnt.value
        return xyz[:n], (out_rgb[:n] if out_rgb is not None else None)

    def set_observation(self, src_depth_cm: torch.Tensor, src_mask: Optional[torch.Tensor],
                        obs_xyz: torch.Tensor, obs_label: Optional[torch.Tensor], sensor_resolution: float,
                        stream=None):
        obs_xyz = obs_xyz.contiguous()
        n = int(obs_xyz.shape[0])
        self._check(self.lib.pcore_set_observation(
            self._h, _ptr(src_depth_cm.contiguous(), torch.int32, "src_depth"),
            _ptr(None if src_mask is None else src_mask.contiguous(), torch.uint8, "src_mask"),
            _ptr(obs_xyz, torch.float32, "obs_xyz") if n else None,
            _ptr(None if obs_label is None else obs_label.contiguous(), torch.int32, "obs_label") if n else None,
            n, float(sensor_resolution), _stream(stream)))

    def set_observation_colors(self, obs_rgb: torch.Tensor, stream=None):
        """Colours (n, 3) uint8 of the observed points given to set_observation, in the same order
        (cost_type 1)."""
        rgb = obs_rgb.contiguous()
        n = int(rgb.shape[0])
        self._check(self.lib.pcore_set_observation_colors(
            self._h, _ptr(rgb, torch.uint8, "obs_rgb") if n else None, n, _stream(stream)))

    # -- per-batch hot path -----------------------------------------------------------------------
    def evaluate(self, poses: torch.Tensor, pose_model: torch.Tensor, pose_label: Optional[torch.Tensor],
                 pose_obs_total: Optional[torch.Tensor], cost_type: int = _native.COST_DEPTH_6DOF,
                 calc_obs_cost: bool = True, stride: int = 8, depth_factor: float = 100.0,
                 sensor_resolution: float = 0.01, occlusion_threshold: float = 1.0,
                 out: Optional[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = None,
                 dbg_zs: Optional[torch.Tensor] = None, color_distance_threshold: float = 15.0, stream=None,
                 select: Optional[Tuple[torch.Tensor, int, int]] = None):
        """Stage COST (do_icp = false).  Returns (rendered_cost, observed_cost, points_diff_cost).  With
        select = (keys, index_base, num_models) the launch also folds every pose's argmin key into `keys`
        (pcore_evaluate_select: the same keys as a following select() call)."""
        n = int(poses.shape[0])
        dev = poses.device
        if out is None:
            out = tuple(torch.empty(n, dtype=torch.float32, device=dev) for _ in range(3))
        rc, oc, df = out
        p = EvalParams(int(cost_type), int(bool(calc_obs_cost)), int(stride), float(depth_factor),
                       float(sensor_resolution), float(occlusion_threshold), float(color_distance_threshold))
        if select is not None:
            keys, index_base, num_models = select
            if dbg_zs is not None:
                raise ValueError("evaluate: dbg_zs and select are exclusive")
            self._check(self.lib.pcore_evaluate_select(
                self._h, _ptr(poses, torch.float32, "poses"), _ptr(pose_model, torch.int32, "pose_model"),
                _ptr(pose_label, torch.int32, "pose_label"), _ptr(pose_obs_total, torch.float32, "pose_obs_total"),
                n, ctypes.byref(p), _ptr(rc, torch.float32, "rc"), _ptr(oc, torch.float32, "oc"),
                _ptr(df, torch.float32, "diff"), int(index_base), int(num_models), _ptr(keys, torch.int64, "keys"),
                _stream(stream)))
            return rc, oc, df
        self._check(self.lib.pcore_evaluate(
            self._h, _ptr(poses, torch.float32, "poses"), _ptr(pose_model, torch.int32, "pose_model"),
            _ptr(pose_label, torch.int32, "pose_label"), _ptr(pose_obs_total, torch.float32, "pose_obs_total"),
            n, ctypes.byref(p), _ptr(rc, torch.float32, "rc"), _ptr(oc, torch.float32, "oc"),
            _ptr(df, torch.float32, "diff"), _ptr(dbg_zs, torch.int32, "dbg_zs"), _stream(stream)))
        return rc, oc, df

    def capture_evaluate(self, poses: torch.Tensor, pose_model: torch.Tensor, pose_label: Optional[torch.Tensor],
                         pose_obs_total: Optional[torch.Tensor], **kw):
        """Stage COST of a fixed-size batch as a HIP graph (torch.cuda.CUDAGraph over the C-ABI launches).
        One warm-up call reserves the scratch, samples the source and picks the LDS tile tier; then the
        launches of one evaluate are captured.  Returns (replay, (rc, oc, diff)): replay() re-scores the batch
        from the tensors' current contents (write new poses into `poses` in place).  For batches small enough
        to be launch-bound (C1: 128 poses); the results equal evaluate()'s.

        The graph bakes in the context state of the capture (sampled source, neighbour grids, scratch
        pointers, tile size).  Any later setup call (upload_meshes, set_camera, set_observation,
        set_observation_colors), a new stride or a larger batch that reallocates scratch changes the
        context's generation (pcore_generation), and replay() then raises PcoreError(PCORE_E_STATE)
        instead of running stale launches: capture again.  The check runs when replay() enqueues the graph, so a
        setup call must be stream-ordered after any replay still in flight."""
        n = int(poses.shape[0])
        out = tuple(torch.empty(n, dtype=torch.float32, device=poses.device) for _ in range(3))
        self.evaluate(poses, pose_model, pose_label, pose_obs_total, out=out, **kw)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            self.evaluate(poses, pose_model, pose_label, pose_obs_total, out=out, **kw)
        gen = self.generation()

        def replay():
            if self.generation() != gen:
                raise PcoreError(_native.PCORE_E_STATE, "captured evaluate graph is stale: the context changed "
                                 "(setup call, new stride or scratch reallocation) since the capture")
            graph.replay()

        return replay, out

    def generation(self) -> int:
        """pcore_generation: changes whenever state a captured evaluate graph depends on may have changed."""
        return int(self.lib.pcore_generation(self._h))

    def evaluate_icp(self, poses: torch.Tensor, pose_model: torch.Tensor, pose_label: Optional[torch.Tensor],
                     pose_obs_total: Optional[torch.Tensor], cost_type: int = _native.COST_DEPTH_6DOF,
                     calc_obs_cost: bool = True, stride: int = 8, depth_factor: float = 100.0,
                     sensor_resolution: float = 0.01, occlusion_threshold: float = 1.0,
                     k: int = _native.ICP_K, max_iterations: int = _native.ICP_MAX_ITER,
                     rotation_epsilon: float = _native.ICP_ROT_EPS,
                     transformation_epsilon: float = _native.ICP_TRANS_EPS, out=None,
                     color_distance_threshold: float = 15.0, stream=None,
                     cycle_exit_window: int = _native.ICP_CYCLE_WINDOW):
        """Stage COST with do_icp = true.  Returns (adjusted poses (N,16), iterations (N,), rc, oc, diff)."""
        n = int(poses.shape[0])
        dev = poses.device
        if out is None:
            out = (torch.empty((n, 16), dtype=torch.float32, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
                   *(torch.empty(n, dtype=torch.float32, device=dev) for _ in range(3)))
        adj, iters, rc, oc, df = out
        p = EvalParams(int(cost_type), int(bool(calc_obs_cost)), int(stride), float(depth_factor),
                       float(sensor_resolution), float(occlusion_threshold), float(color_distance_threshold))
        ip = IcpParams(int(k), int(max_iterations), float(rotation_epsilon), float(transformation_epsilon),
                       int(cycle_exit_window))
        self._check(self.lib.pcore_evaluate_icp(
            self._h, _ptr(poses, torch.float32, "poses"), _ptr(pose_model, torch.int32, "pose_model"),
            _ptr(pose_label, torch.int32, "pose_label"), _ptr(pose_obs_total, torch.float32, "pose_obs_total"),
            n, ctypes.byref(p), ctypes.byref(ip), _ptr(adj, torch.float32, "adjusted_poses"),
            _ptr(iters, torch.int32, "iterations"), _ptr(rc, torch.float32, "rc"), _ptr(oc, torch.float32, "oc"),
            _ptr(df, torch.float32, "diff"), _stream(stream)))
        return adj, iters, rc, oc, df

    def render(self, poses: torch.Tensor, pose_model: torch.Tensor, pose_label: Optional[torch.Tensor],
               occlusion_threshold: float = 1.0, out: Optional[torch.Tensor] = None, color: bool = False,
               out_color: Optional[torch.Tensor] = None, stream=None):
        """Stage RENDER: (N, H, W) int32 z-buffers in cm; with color=True also the reference's result_color planes,
        returned as (depth, color (3, N, H, W) uint8 red / green / blue)."""
        n = int(poses.shape[0])
        if out is None:
            out = torch.empty((n, self.height, self.width), dtype=torch.int32, device=poses.device)
        if color and out_color is None:
            out_color = torch.empty((3, n, self.height, self.width), dtype=torch.uint8, device=poses.device)
        self._check(self.lib.pcore_render(
            self._h, _ptr(poses, torch.float32, "poses"), _ptr(pose_model, torch.int32, "pose_model"),
            _ptr(pose_label, torch.int32, "pose_label"), n, float(occlusion_threshold),
            _ptr(out, torch.int32, "out"), _ptr(out_color, torch.uint8, "out_color") if color else None,
            _stream(stream)))
        return (out, out_color) if color else out

    def stats(self, reset: bool = False) -> dict:
        """pcore_get_stats: the reference's gpu_stats of the last evaluate_icp (waits for its GICP stage)."""
        st = _native.GpuStats()
        self._check(self.lib.pcore_get_stats(self._h, ctypes.byref(st), int(bool(reset))))
        return {"icp_runtime": st.icp_runtime, "peak_memory_usage": st.peak_memory_usage, "gicp_ms": st.gicp_ms,
                "icp_chunks": st.icp_chunks, "gicp_iterations": st.gicp_iterations,
                "gicp_iterations_run": st.gicp_iterations_run, "gicp_cycle_exits": st.gicp_cycle_exits}

    def gicp_help_stats(self) -> dict:
        """pcore_debug_gicp_help_stats: the last evaluate_icp's GICP help board counters."""
        out = (ctypes.c_int64 * 4)()
        self._check(self.lib.pcore_debug_gicp_help_stats(self._h, out))
        return {"helper_rounds": int(out[0]), "owner_timeouts": int(out[1]), "helper_giveups": int(out[2]),
                "poses_enlisted": int(out[3])}

    def tile_info(self) -> dict:
        """pcore_get_tile_info: the fused window launch's tile tier and the last published window histogram."""
        ti = _native.TileInfo()
        self._check(self.lib.pcore_get_tile_info(self._h, ctypes.byref(ti)))
        n = ti.num_tiers
        return {"tier": ti.tier, "tcap": ti.tcap, "seq": ti.seq, "edge": list(ti.edge[:n]),
                "wgs_per_cu": list(ti.wgs_per_cu[:n]), "hist": list(ti.hist[:n + 1]), "chunked": ti.chunked}

    def depth_to_cloud(self, depth: torch.Tensor, stride: int, depth_factor: float,
                       label_mask: Optional[torch.Tensor] = None, pose_label: Optional[torch.Tensor] = None,
                       stream=None, color_planes: Optional[torch.Tensor] = None, dc_index: bool = False):
        """Stage CLOUD (compute_point_clouds): returns (xyz (P,3), pose (P,), label (P,)); with `color_planes` (the
        rendered colour planes, uint8 (3, N, H, W): `render(..., color=True)`'s second output) also the points'
        colours (3, P) -- renderer.cu's result_cloud_color -- and with dc_index=True also result_dc_index (N, H, W)
        int32 (pcore_depth_to_cloud_ex), appended in that order."""
        if depth.dim() == 2:
            depth = depth.unsqueeze(0)
        n, h, w = depth.shape
        cap = n * ((w + stride - 1) // stride) * ((h + stride - 1) // stride)
        dev = depth.device
        xyz = torch.empty((max(cap, 1), 3), dtype=torch.float32, device=dev)
        pose = torch.empty((max(cap, 1),), dtype=torch.int32, device=dev)
        lab = torch.empty((max(cap, 1),), dtype=torch.int32, device=dev)
        cnt = ctypes.c_int32(0)
        extra = color_planes is not None or dc_index
        if not extra:
            self._check(self.lib.pcore_depth_to_cloud(
                self._h, _ptr(depth.contiguous(), torch.int32, "depth"), n, w, h, stride, float(depth_factor),
                _ptr(label_mask, torch.uint8, "label_mask"), _ptr(pose_label, torch.int32, "pose_label"),
                _ptr(xyz, torch.float32, "xyz"), _ptr(pose, torch.int32, "pose"), _ptr(lab, torch.int32, "label"),
                cap, ctypes.byref(cnt), _stream(stream)))
            k = cnt.value
            return xyz[:k], pose[:k], lab[:k]
        planes = None
        col = None
        if color_planes is not None:
            planes = color_planes.contiguous()
            if tuple(planes.shape) != (3, n, h, w):
                raise ValueError(f"color_planes must be (3, {n}, {h}, {w}), got {tuple(planes.shape)}")
            col = torch.empty((3, max(cap, 1)), dtype=torch.uint8, device=dev)
        dc = torch.empty((n, h, w), dtype=torch.int32, device=dev) if dc_index else None
        self._check(self.lib.pcore_depth_to_cloud_ex(
            self._h, _ptr(depth.contiguous(), torch.int32, "depth"), n, w, h, stride, float(depth_factor),
            _ptr(label_mask, torch.uint8, "label_mask"), _ptr(pose_label, torch.int32, "pose_label"),
            _ptr(planes, torch.uint8, "color_planes"), _ptr(xyz, torch.float32, "xyz"), _ptr(pose, torch.int32, "pose"),
            _ptr(lab, torch.int32, "label"), _ptr(col, torch.uint8, "color"), _ptr(dc, torch.int32, "dc_index"),
            max(cap, 1) if col is not None else cap, ctypes.byref(cnt), _stream(stream)))
        k = cnt.value
        out = [xyz[:k], pose[:k], lab[:k]]
        if col is not None:
            out.append(col[:, :k])
        if dc is not None:
            out.append(dc)
        return tuple(out)

    def select(self, rc: torch.Tensor, oc: torch.Tensor, pose_model: torch.Tensor, num_models: int,
               index_base: int = 0, keys: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        """Per-model argmin keys (int64), folded into `keys` (initialised to PCORE_KEY_NONE)."""
        if keys is None:
            keys = torch.full((num_models,), _native.PCORE_KEY_NONE, dtype=torch.int64, device=rc.device)
        self._check(self.lib.pcore_select(
            self._h, _ptr(rc, torch.float32, "rc"), _ptr(oc, torch.float32, "oc"),
            _ptr(pose_model, torch.int32, "pose_model"), int(rc.shape[0]), int(index_base), int(num_models),
            _ptr(keys, torch.int64, "keys"), _stream(stream)))
        return keys

    def count_within(self, queries: torch.Tensor, labels: torch.Tensor, radius_sq: torch.Tensor,
                     out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        """IsValidPose neighbour counts (pcore_count_within): for every query (n x 3 float32), the points of its
        observed label segment strictly within sqrt(radius_sq) (float32 per query), PCL radiusSearch semantics."""
        n = int(queries.shape[0])
        if out is None:
            out = torch.empty(n, dtype=torch.int32, device=queries.device)
        self._check(self.lib.pcore_count_within(
            self._h, _ptr(queries.contiguous(), torch.float32, "queries"), _ptr(labels.contiguous(), torch.int32, "labels"),
            _ptr(radius_sq.contiguous(), torch.float32, "radius_sq"), n, _ptr(out, torch.int32, "counts"),
            _stream(stream)))
        return out

    def state_poses(self, states: torch.Tensor, model: torch.Tensor, cam_from_world, preprocess: torch.Tensor,
                    out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        """The states' search poses (pcore_state_poses): init_from_eigen(cam_from_world * T(state) *
        preprocess[model], 100) for states (n x 7 float64: x y z qx qy qz qw), as N x 16 float32."""
        n = int(states.shape[0])
        if out is None:
            out = torch.empty((n, 16), dtype=torch.float32, device=states.device)
        cam = (ctypes.c_double * 16)(*[float(v) for v in np.asarray(cam_from_world, np.float64).reshape(16)])
        k = int(preprocess.shape[0])
        self._check(self.lib.pcore_state_poses(
            self._h, _ptr(states.contiguous(), torch.float64, "states"), _ptr(model.contiguous(), torch.int32, "model"),
            cam, _ptr(preprocess.contiguous(), torch.float64, "preprocess"), k, n, _ptr(out, torch.float32, "poses"),
            _stream(stream)))
        return out


class PoseLanes:
    """Batches in flight on one device: `lanes` independent contexts, each with its own HIP stream.

    A stage-COST launch ends with a drain (its last workgroups leave CUs idle) and starts with a fill in which
    every workgroup runs the same phase at once; on one stream the next batch waits for the drain.  Consecutive
    batches submitted to consecutive lanes overlap one batch's drain with the next one's fill (C2, 10k poses
    per batch: 0.40 -> 0.36 ms per batch with two lanes; tools/pipeline_probe.py).  Every lane holds the same
    meshes, camera and observation (setup calls go to all of them) and its own scratch, so lanes never share
    per-batch state, and each lane's results equal a single context's bit for bit.

    Work on lane i runs on streams[i]: run the whole step (evaluate, select, anything reading its outputs) under
    `with torch.cuda.stream(lanes.streams[i])`, or pass stream=.  Inputs written on another stream must be
    ordered before the lane's stream (lanes.streams[i].wait_stream(...)); lane i's output buffers are reused
    only by lane i, so stream order protects them."""

    def __init__(self, device: int = 0, lanes: int = 2):
        if lanes < 1:
            raise ValueError("lanes must be >= 1")
        self.cores = [PoseCore(device) for _ in range(lanes)]
        dev = torch.device("cuda", int(device))
        self.streams = [torch.cuda.Stream(device=dev) for _ in range(lanes)]

    def __len__(self):
        return len(self.cores)

    def __getitem__(self, i: int) -> Tuple[PoseCore, torch.cuda.Stream]:
        return self.cores[i], self.streams[i]

    def upload_meshes(self, *a, **kw):
        for c in self.cores:
            c.upload_meshes(*a, **kw)

    def set_camera(self, *a, **kw):
        for c in self.cores:
            c.set_camera(*a, **kw)

    def set_observation(self, *a, **kw):
        for c in self.cores:
            c.set_observation(*a, **kw)

    def set_observation_colors(self, *a, **kw):
        for c in self.cores:
            c.set_observation_colors(*a, **kw)

    @classmethod
    def replicate(cls, core: "PoseCore", scene_setup, lanes: int = 2) -> "PoseLanes":
        """Lanes whose lane 0 is an existing, set-up context; scene_setup(c) repeats its setup on a new one."""
        if lanes < 1:
            raise ValueError("lanes must be >= 1")
        self = cls.__new__(cls)
        self.cores = [core] + [PoseCore(core.device) for _ in range(lanes - 1)]
        dev = torch.device("cuda", core.device)
        self.streams = [torch.cuda.Stream(device=dev) for _ in range(lanes)]
        for c in self.cores[1:]:
            scene_setup(c)
        return self


def decode_keys(keys) -> Tuple[np.ndarray, np.ndarray]:
    """Per-model key -> (best cost, best global index); (INT_MAX, -1) where no pose qualified."""
    k = np.asarray(keys.cpu() if isinstance(keys, torch.Tensor) else keys, dtype=np.int64)
    none = k == _native.PCORE_KEY_NONE
    hi = (k >> 31).astype(np.uint64).astype(np.uint32)
    cost = (hi ^ np.uint32(0x80000000)).view(np.int32).astype(np.int32)
    idx = (k & 0x7FFFFFFF).astype(np.int64)
    cost = np.where(none, np.int32(2**31 - 1), cost)
    idx = np.where(none, -1, idx)
    return cost, idx


def encode_key(cost: int, index: int) -> int:
    """The int64 selection key of pcore_select (include/pcore.h): ((cost ^ 0x80000000) << 31) | index."""
    if cost == 2**31 - 1 and index < 0:
        return _native.PCORE_KEY_NONE
    hi = (int(cost) & 0xFFFFFFFF) ^ 0x80000000
    return (hi << 31) | (int(index) & 0x7FFFFFFF)
