"""ctypes binding of libpcore.so (include/pcore.h).

The product path has no CPU fallback: if the HIP library is missing or fails to load, importing the
binding raises.  `load()` never builds implicitly on a machine without hipcc.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import build as _build

PCORE_OK = 0
PCORE_E_INVALID_ARG = 1
PCORE_E_HIP = 2
PCORE_E_OOM = 3
PCORE_E_STATE = 4
PCORE_KEY_NONE = 0x7FFFFFFFFFFFFFFF

COST_DEPTH_3DOF = 0
COST_RGBD_3DOF = 1
COST_DEPTH_6DOF = 2

# every symbol declared in include/pcore.h
EXPORTED_SYMBOLS = (
    "pcore_create", "pcore_destroy", "pcore_last_error", "pcore_abi_version", "pcore_upload_meshes",
    "pcore_set_camera", "pcore_observed_cloud", "pcore_set_observation", "pcore_evaluate", "pcore_evaluate_icp",
    "pcore_render",
    "pcore_depth_to_cloud", "pcore_select", "pcore_pose_distances",
    "pcore_observed_cloud_bounded", "pcore_set_observation_colors", "pcore_generation", "pcore_get_stats",
    "pcore_count_within", "pcore_state_poses", "pcore_evaluate_select", "pcore_get_tile_info", "pcore_debug_lm_solve",
    "pcore_debug_covariances", "pcore_debug_covariances_cloud", "pcore_debug_gicp_help_stats", "pcore_depth_to_cloud_ex",
)


class PcoreError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"pcore error {code}: {msg}")
        self.code = code


class Camera(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("fx", ctypes.c_float),
                ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("proj", ctypes.c_float * 16)]


class EvalParams(ctypes.Structure):
    _fields_ = [("cost_type", ctypes.c_int32), ("calc_obs_cost", ctypes.c_int32), ("stride", ctypes.c_int32),
                ("depth_factor", ctypes.c_float), ("sensor_resolution", ctypes.c_float),
                ("occlusion_threshold", ctypes.c_float), ("color_distance_threshold", ctypes.c_float)]


class GpuStats(ctypes.Structure):
    """pcore_gpu_stats (include/pcore.h; the reference's gpu_stats, model.h:24-27)."""
    _fields_ = [("icp_runtime", ctypes.c_float), ("peak_memory_usage", ctypes.c_double), ("gicp_ms", ctypes.c_float),
                ("icp_chunks", ctypes.c_int32), ("gicp_iterations", ctypes.c_int64),
                ("gicp_iterations_run", ctypes.c_int64), ("gicp_cycle_exits", ctypes.c_int64)]


MAX_TILE_TIERS = 8


class TileInfo(ctypes.Structure):
    """pcore_tile_info (include/pcore.h): the fused window launch's LDS tile and its window histogram."""
    _fields_ = [("num_tiers", ctypes.c_int32), ("tier", ctypes.c_int32), ("tcap", ctypes.c_int32),
                ("seq", ctypes.c_int32), ("edge", ctypes.c_int32 * MAX_TILE_TIERS),
                ("wgs_per_cu", ctypes.c_int32 * MAX_TILE_TIERS), ("hist", ctypes.c_int32 * (MAX_TILE_TIERS + 1)),
                ("chunked", ctypes.c_int32)]


class IcpParams(ctypes.Structure):
    _fields_ = [("k_correspondences", ctypes.c_int32), ("max_iterations", ctypes.c_int32),
                ("rotation_epsilon", ctypes.c_double), ("transformation_epsilon", ctypes.c_double),
                ("cycle_exit_window", ctypes.c_int32)]


# renderer.cu:1696-1699
ICP_K = 10
ICP_MAX_ITER = 150
# renderer.cu:1698-1699 declares both as float and passes them to set_*_epsilon(double): the float values widened
ICP_ROT_EPS = float(np.float32(2e-3))
ICP_TRANS_EPS = float(np.float32(5e-4))
# the GICP cycle exit's window (include/pcore.h PCORE_GICP_CYCLE_WINDOW; 0 = off)
ICP_CYCLE_WINDOW = 8

_lib = None


def library_path() -> str:
    return _build.LIB


def load(auto_build: bool = True) -> ctypes.CDLL:
    """Load libpcore.so (building it in-tree first when hipcc is available and sources are newer)."""
    global _lib
    if _lib is not None:
        return _lib
    override = os.environ.get("PCORE_LIB")  # A/B profiling of alternative builds of the same sources
    if override:
        auto_build = False
    if auto_build:
        try:
            if _build.needs_build():
                _build.build()
        except (RuntimeError, OSError) as e:  # no hipcc on this machine: fall through to the prebuilt .so
            if not os.path.exists(_build.LIB):
                raise RuntimeError(f"libpcore.so is missing and cannot be built: {e}") from e
    path = override or _build.LIB
    if not os.path.exists(path):
        raise RuntimeError(f"libpcore.so not found at {path}; run `python -m perception_amd.build`")
    L = ctypes.CDLL(path)
    vp, i32, i64, f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float
    L.pcore_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.pcore_destroy.argtypes = [vp]
    L.pcore_destroy.restype = None
    L.pcore_last_error.argtypes = [vp]
    L.pcore_last_error.restype = ctypes.c_char_p
    L.pcore_abi_version.argtypes = []
    L.pcore_upload_meshes.argtypes = [vp, vp, vp, i32, vp, i32]
    L.pcore_set_camera.argtypes = [vp, ctypes.POINTER(Camera)]
    L.pcore_observed_cloud.argtypes = [vp, vp, vp, i32, i32, i32, f32, vp, vp, i32, ctypes.POINTER(i32), vp]
    L.pcore_set_observation.argtypes = [vp, vp, vp, vp, vp, i32, f32, vp]
    L.pcore_evaluate.argtypes = [vp, vp, vp, vp, vp, i32, ctypes.POINTER(EvalParams), vp, vp, vp, vp, vp]
    L.pcore_evaluate_icp.argtypes = [vp, vp, vp, vp, vp, i32, ctypes.POINTER(EvalParams), ctypes.POINTER(IcpParams),
                                     vp, vp, vp, vp, vp, vp]
    L.pcore_render.argtypes = [vp, vp, vp, vp, i32, f32, vp, vp, vp]
    L.pcore_get_stats.argtypes = [vp, ctypes.POINTER(GpuStats), i32]
    if hasattr(L, "pcore_get_tile_info"):  # diagnostics / test hooks: absent from older A/B builds (PCORE_LIB)
        L.pcore_get_tile_info.argtypes = [vp, ctypes.POINTER(TileInfo)]
    if hasattr(L, "pcore_debug_lm_solve"):
        L.pcore_debug_lm_solve.argtypes = [vp, vp, vp, i32, vp]
    if hasattr(L, "pcore_debug_covariances"):
        L.pcore_debug_covariances.argtypes = [vp, vp, vp, i32, i32, vp, vp]
    if hasattr(L, "pcore_debug_gicp_help_stats"):
        L.pcore_debug_gicp_help_stats.argtypes = [vp, vp]
    if hasattr(L, "pcore_debug_covariances_cloud"):
        f32 = ctypes.c_float
        L.pcore_debug_covariances_cloud.argtypes = [vp, vp, i32, i32, f32, f32, f32, f32, i32, vp, vp]
    if hasattr(L, "pcore_depth_to_cloud_ex"):
        L.pcore_depth_to_cloud_ex.argtypes = [vp, vp, i32, i32, i32, i32, f32, vp, vp, vp, vp, vp, vp, vp, vp, i32,
                                              ctypes.POINTER(i32), vp]
    L.pcore_depth_to_cloud.argtypes = [vp, vp, i32, i32, i32, i32, f32, vp, vp, vp, vp, vp, i32,
                                       ctypes.POINTER(i32), vp]
    L.pcore_select.argtypes = [vp, vp, vp, vp, i32, i64, i32, vp, vp]
    L.pcore_pose_distances.argtypes = [vp, vp, i32, vp, vp, i32, vp, vp, vp]
    L.pcore_set_observation_colors.argtypes = [vp, vp, i32, vp]
    L.pcore_observed_cloud_bounded.argtypes = [vp, vp, vp, i32, i32, i32, f32, vp, vp, vp, vp, i32,
                                               ctypes.POINTER(i32), vp]
    L.pcore_generation.argtypes = [vp]
    L.pcore_evaluate_select.argtypes = [vp, vp, vp, vp, vp, i32, ctypes.POINTER(EvalParams), vp, vp, vp, i64, i32,
                                        vp, vp]
    L.pcore_count_within.argtypes = [vp, vp, vp, vp, i32, vp, vp]
    L.pcore_state_poses.argtypes = [vp, vp, vp, ctypes.POINTER(ctypes.c_double), vp, i32, i32, vp, vp]
    for name in EXPORTED_SYMBOLS:
        if name not in ("pcore_destroy", "pcore_last_error", "pcore_generation") and hasattr(L, name):
            getattr(L, name).restype = ctypes.c_int
    L.pcore_generation.restype = ctypes.c_uint64
    _lib = L
    return L
