"""CPU oracle for the render-and-compare hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this package.  The
product package (perception_amd) never imports, links or calls it.

This is a literal restatement of the reference's CUDA/host code (file:line citations in
pcore_oracle.cpp).  Parity against the reference *binary* is unpinned: the reference path cannot be
built here and holds no golden vectors for this path ("Oracle").
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")


def build() -> str:
    """Compile oracle/build/liboracle.so with the oracle's Makefile (g++, no FMA contraction)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def _opt(ptype):
    """ndpointer that also accepts None (NULL)."""

    class _Opt(ptype):
        @classmethod
        def from_param(cls, obj):
            if obj is None:
                return None
            return super().from_param(obj)

    return _Opt


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        c_int, c_float = ctypes.c_int, ctypes.c_float
        L.orc_compute_proj.argtypes = [c_float] * 4 + [c_int, c_int, c_float, c_float, _f32p]
        L.orc_render_depth.argtypes = [_f32p, c_int, _i32p, c_int, _f32p, _i32p, _opt(_i32p), c_int,
                                       c_int, c_int, _f32p, _i32p, _opt(_u8p), c_float, _i32p, c_int]
        L.orc_depth_to_cloud.restype = c_int
        L.orc_depth_to_cloud.argtypes = [_i32p, c_int, c_int, c_int, c_int, c_float, c_float, c_float, c_float,
                                         c_float, _opt(_u8p), _opt(_i32p), _f32p, _opt(_i32p), _opt(_i32p), c_int]
        L.orc_knn1.argtypes = [_f32p, _opt(_i32p), c_int, _f32p, c_int, _opt(_i32p), _opt(_i32p), c_int,
                               _f32p, _i32p]
        L.orc_costs.argtypes = [c_int, c_int, c_int, c_float, _f32p, _i32p, _i32p, c_int, c_int,
                                _opt(_f32p), _f32p, _f32p, _f32p]
        L.orc_select.argtypes = [c_int, _f32p, _f32p, _i32p, c_int, ctypes.c_int64, _i32p, _i64p]
        L.orc_evaluate.argtypes = [_f32p, c_int, _i32p, c_int, _f32p, _i32p, _opt(_i32p), c_int, c_int, c_int,
                                   _f32p, _i32p, _opt(_u8p), c_float, c_int, c_float, c_float, c_float, c_float,
                                   c_float, _f32p, c_int, _opt(_i32p), _opt(_i32p), c_int, _opt(_f32p), c_int,
                                   c_int, c_float, _f32p, _f32p, _f32p, c_int]
        _lib = L
    return _lib


def _c(a, dt):
    return None if a is None else np.ascontiguousarray(a, dtype=dt)


def compute_proj(fx, fy, cx, cy, width, height, near=10.0, far=10000.0) -> np.ndarray:
    out = np.zeros(16, np.float32)
    lib().orc_compute_proj(fx, fy, cx, cy, width, height, near, far, out)
    return out


def render_depth(tris, tris_model_count, poses, pose_model, pose_label, width, height, proj,
                 src_depth, src_mask, occlusion_threshold=1.0, nthreads=0) -> np.ndarray:
    tris = _c(tris, np.float32).reshape(-1)
    poses = _c(poses, np.float32).reshape(-1)
    n = poses.size // 16
    out = np.empty((n, height, width), np.int32)
    lib().orc_render_depth(tris, tris.size // 9, _c(tris_model_count, np.int32), len(tris_model_count), poses,
                           _c(pose_model, np.int32), _c(pose_label, np.int32), n, width, height,
                           _c(proj, np.float32), _c(src_depth, np.int32).reshape(-1),
                           None if src_mask is None else _c(src_mask, np.uint8).reshape(-1),
                           float(occlusion_threshold), out.reshape(-1), nthreads)
    return out


def render_depth_color(tris, tri_rgb, tris_model_count, poses, pose_model, pose_label, width, height, proj,
                       src_depth, src_mask, occlusion_threshold=1.0, nthreads=0):
    """Stage RENDER with colours: (depth (N, H, W) int32, colour (3, N, H, W) uint8 red / green / blue planes, the
    layout of the reference's result_color)."""
    L = lib()
    if not getattr(L, "_rgb_typed", False):
        L.orc_render_depth_color.argtypes = [_f32p, ctypes.c_int, _opt(_u8p), _i32p, ctypes.c_int, _f32p, _i32p,
                                             _opt(_i32p), ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p, _i32p,
                                             _opt(_u8p), ctypes.c_float, _i32p, _u8p, ctypes.c_int]
        L._rgb_typed = True
    tris = _c(tris, np.float32).reshape(-1)
    poses = _c(poses, np.float32).reshape(-1)
    n = poses.size // 16
    out = np.empty((n, height, width), np.int32)
    col = np.empty((n, 3, height, width), np.uint8)
    L.orc_render_depth_color(tris, tris.size // 9, None if tri_rgb is None else _c(tri_rgb, np.uint8).reshape(-1),
                             _c(tris_model_count, np.int32), len(tris_model_count), poses, _c(pose_model, np.int32),
                             _c(pose_label, np.int32), n, width, height, _c(proj, np.float32),
                             _c(src_depth, np.int32).reshape(-1),
                             None if src_mask is None else _c(src_mask, np.uint8).reshape(-1),
                             float(occlusion_threshold), out.reshape(-1), col.reshape(-1), nthreads)
    return out, np.ascontiguousarray(col.transpose(1, 0, 2, 3))


def depth_to_cloud(depth, stride, cx, cy, fx, fy, depth_factor, label_mask=None, pose_label=None):
    """Returns (xyz (P,3) f32, pose (P,) i32, label (P,) i32) in the reference's compaction order."""
    depth = _c(depth, np.int32)
    n, h, w = depth.shape if depth.ndim == 3 else (1,) + depth.shape
    cap = n * ((h + stride - 1) // stride) * ((w + stride - 1) // stride)
    xyz = np.zeros((max(cap, 1), 3), np.float32)
    pose = np.zeros(max(cap, 1), np.int32)
    lab = np.zeros(max(cap, 1), np.int32)
    cnt = lib().orc_depth_to_cloud(depth.reshape(-1), n, w, h, stride, cx, cy, fx, fy, depth_factor,
                                   None if label_mask is None else _c(label_mask, np.uint8).reshape(-1),
                                   _c(pose_label, np.int32), xyz.reshape(-1), pose, lab, cap)
    return xyz[:cnt].copy(), pose[:cnt].copy(), lab[:cnt].copy()


def depth_to_cloud_bounded(depth, stride, cx, cy, fx, fy, depth_factor, cam_to_world=None, bounds=None, rgb=None):
    """3-DoF observed cloud: (xyz (P,3) f32 camera frame, rgb (P,3) u8 or None)."""
    depth = _c(depth, np.int32)
    h, w = depth.shape
    cap = ((h + stride - 1) // stride) * ((w + stride - 1) // stride)
    xyz = np.zeros((max(cap, 1), 3), np.float32)
    out_rgb = np.zeros((max(cap, 1), 3), np.uint8)
    L = lib()
    L.orc_depth_to_cloud_bounded.restype = ctypes.c_int
    L.orc_depth_to_cloud_bounded.argtypes = [_i32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                             ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                             _opt(_f32p), _opt(np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")),
                                             _opt(_u8p), _f32p, _u8p, ctypes.c_int]
    cnt = L.orc_depth_to_cloud_bounded(
        depth.reshape(-1), w, h, stride, cx, cy, fx, fy, depth_factor,
        None if cam_to_world is None else _c(cam_to_world, np.float32).reshape(-1),
        None if bounds is None else _c(bounds, np.float64).reshape(-1),
        None if rgb is None else _c(rgb, np.uint8).reshape(-1), xyz.reshape(-1), out_rgb.reshape(-1), cap)
    return xyz[:cnt].copy(), (out_rgb[:cnt].copy() if rgb is not None else None)


def knn1(r_xyz, r_label, o_xyz, label_start=None, label_end=None):
    r_xyz = _c(r_xyz, np.float32).reshape(-1, 3)
    o_xyz = _c(o_xyz, np.float32).reshape(-1, 3)
    nr = r_xyz.shape[0]
    d2 = np.zeros(max(nr, 1), np.float32)
    idx = np.zeros(max(nr, 1), np.int32)
    nl = 0 if label_start is None else len(label_start)
    lib().orc_knn1(r_xyz.reshape(-1) if nr else np.zeros(3, np.float32), _c(r_label, np.int32), nr,
                   o_xyz.reshape(-1) if o_xyz.size else np.zeros(3, np.float32), o_xyz.shape[0],
                   _c(label_start, np.int32), _c(label_end, np.int32), nl, d2, idx)
    return d2[:nr], idx[:nr]


def costs(num_poses, cost_type, calc_obs, sensor_resolution, d2, idx, r_pose, num_o, pose_obs_total):
    rc = np.zeros(num_poses, np.float32)
    oc = np.zeros(num_poses, np.float32)
    df = np.zeros(num_poses, np.float32)
    d2 = _c(d2, np.float32)
    lib().orc_costs(num_poses, cost_type, int(calc_obs), sensor_resolution,
                    d2 if d2.size else np.zeros(1, np.float32), _c(idx, np.int32) if len(idx) else np.zeros(1, np.int32),
                    _c(r_pose, np.int32) if len(r_pose) else np.zeros(1, np.int32), len(d2), num_o,
                    _c(pose_obs_total, np.float32), rc, oc, df)
    return rc, oc, df


def select(rc, oc, pose_model, num_models, index_base=0):
    best_cost = np.zeros(num_models, np.int32)
    best_idx = np.zeros(num_models, np.int64)
    lib().orc_select(len(rc), _c(rc, np.float32), _c(oc, np.float32), _c(pose_model, np.int32), num_models,
                     index_base, best_cost, best_idx)
    return best_cost, best_idx


def evaluate(tris, tris_model_count, poses, pose_model, pose_label, width, height, proj, src_depth, src_mask,
             occlusion_threshold, stride, cx, cy, fx, fy, depth_factor, o_xyz, label_start, label_end,
             pose_obs_total, cost_type, calc_obs, sensor_resolution, nthreads=0):
    tris = _c(tris, np.float32).reshape(-1)
    poses = _c(poses, np.float32).reshape(-1)
    n = poses.size // 16
    o_xyz = _c(o_xyz, np.float32).reshape(-1)
    rc = np.zeros(n, np.float32)
    oc = np.zeros(n, np.float32)
    df = np.zeros(n, np.float32)
    nl = 0 if label_start is None else len(label_start)
    lib().orc_evaluate(tris, tris.size // 9, _c(tris_model_count, np.int32), len(tris_model_count), poses,
                       _c(pose_model, np.int32), _c(pose_label, np.int32), n, width, height, _c(proj, np.float32),
                       _c(src_depth, np.int32).reshape(-1),
                       None if src_mask is None else _c(src_mask, np.uint8).reshape(-1), float(occlusion_threshold),
                       stride, cx, cy, fx, fy, depth_factor,
                       o_xyz if o_xyz.size else np.zeros(3, np.float32), o_xyz.size // 3,
                       _c(label_start, np.int32), _c(label_end, np.int32), nl, _c(pose_obs_total, np.float32),
                       cost_type, int(calc_obs), sensor_resolution, rc, oc, df, nthreads)
    return rc, oc, df


_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")


def _gicp_lib():
    L = lib()
    if not getattr(L, "_gicp_typed", False):
        c_int, c_float, c_double = ctypes.c_int, ctypes.c_float, ctypes.c_double
        L.orc_covariances.argtypes = [_f32p, c_int, c_int, _f64p]
        L.orc_gicp.restype = c_int
        L.orc_gicp.argtypes = [_f32p, _f64p, c_int, _f32p, _f64p, c_int, c_int, c_double, c_double, c_int, _f64p]
        L.orc_concat_pose.argtypes = [_f64p, _f32p, _f32p]
        L.orc_evaluate_icp.argtypes = [_f32p, c_int, _i32p, c_int, _f32p, _i32p, _opt(_i32p), c_int, c_int, c_int,
                                       _f32p, _i32p, _opt(_u8p), c_float, c_int, c_float, c_float, c_float, c_float,
                                       c_float, _f32p, _f64p, c_int, _opt(_i32p), _opt(_i32p), c_int, _opt(_f32p),
                                       c_int, c_int, c_float, c_int, c_int, c_double, c_double, c_int, _f32p,
                                       _opt(_i32p), _f32p, _f32p, _f32p, c_int]
        L.orc_gicp_trace.restype = c_int
        L.orc_gicp_trace.argtypes = [_f32p, _f64p, c_int, _f32p, _f64p, c_int, c_int, c_double, c_double, c_int,
                                     _f64p, _opt(_f64p), _opt(_i32p), c_int]
        L.orc_gicp_lm_solve_ldlt.argtypes = [_f64p, c_double, _f64p]
        L.orc_gicp_linearize.argtypes = [_f32p, _f64p, c_int, _f32p, _f64p, c_int, _f64p, c_int, _i32p, _f64p]
        L.orc_gicp_se3_exp.argtypes = [_f64p, _f64p]
        L.orc_gicp_lm_solve.argtypes = [_f64p, c_double, _f64p]
        L.orc_sin_d.restype = c_double
        L.orc_sin_d.argtypes = [c_double]
        L.orc_cos_d.restype = c_double
        L.orc_cos_d.argtypes = [c_double]
        for fn in (L.orc_cube_rn, L.orc_lm_gain):
            fn.restype = c_double
            fn.argtypes = [c_double]
        L.orc_gicp_nn.argtypes = [_f32p, c_int, _f32p, c_int, _i32p]
        L._gicp_typed = True
    return L


GICP_K = 10            # renderer.cu:1697 k_correspondences_
GICP_MAX_ITER = 150    # renderer.cu:1696
GICP_ROT_EPS = float(np.float32(2e-3))    # renderer.cu:1698 (a float widened to double)
GICP_TRANS_EPS = float(np.float32(5e-4))  # renderer.cu:1699 (a float widened to double)
GICP_CYCLE_WINDOW = 8  # the spec's cycle exit window W (pcore_gicp_math.h kCycleWindow; 0 = run the iterations out)


def covariances(xyz, k=GICP_K):
    xyz = _c(xyz, np.float32).reshape(-1, 3)
    out = np.zeros((max(len(xyz), 1), 6), np.float64)
    if len(xyz):
        _gicp_lib().orc_covariances(xyz.reshape(-1), len(xyz), k, out.reshape(-1))
    return out[:len(xyz)]


def gicp(src, src_cov, tgt, tgt_cov, max_iter=GICP_MAX_ITER, rot_eps=GICP_ROT_EPS, trans_eps=GICP_TRANS_EPS,
         cycle_window=GICP_CYCLE_WINDOW):
    src = _c(src, np.float32).reshape(-1, 3)
    tgt = _c(tgt, np.float32).reshape(-1, 3)
    T = np.zeros(16, np.float64)
    z3, z6 = np.zeros(3, np.float32), np.zeros(6, np.float64)
    it = _gicp_lib().orc_gicp(src.reshape(-1) if len(src) else z3, _c(src_cov, np.float64).reshape(-1) if len(src) else z6,
                              len(src), tgt.reshape(-1) if len(tgt) else z3,
                              _c(tgt_cov, np.float64).reshape(-1) if len(tgt) else z6, len(tgt), max_iter, rot_eps,
                              trans_eps, int(cycle_window), T)
    return T.reshape(4, 4), it


def gicp_trace(src, src_cov, tgt, tgt_cov, max_iter=GICP_MAX_ITER, rot_eps=GICP_ROT_EPS, trans_eps=GICP_TRANS_EPS,
               cycle_window=0, solver="schur"):
    """orc_gicp with its per-iteration trace: (T, iterations reported, trace (executed iterations, 16): R (9), t (3)
    after each iteration, the lambda of its first trial, its number of trials, flags (1: lambda inert, 2: accepted
    with rho >= 1/2), the LM status).  The cycle exit is off unless cycle_window > 0.  solver "schur" is the spec's
    damped solve, "ldlt" Eigen's pivoted LDLT as fast_gicp uses it (a test reference)."""
    src = _c(src, np.float32).reshape(-1, 3)
    tgt = _c(tgt, np.float32).reshape(-1, 3)
    T = np.zeros(16, np.float64)
    tr = np.zeros((max_iter, 16), np.float64)
    ex = np.zeros(1, np.int32)
    it = _gicp_lib().orc_gicp_trace(src.reshape(-1), _c(src_cov, np.float64).reshape(-1), len(src), tgt.reshape(-1),
                                    _c(tgt_cov, np.float64).reshape(-1), len(tgt), max_iter, rot_eps, trans_eps,
                                    int(cycle_window), T, tr.reshape(-1), ex, {"schur": 0, "ldlt": 1}[solver])
    return T.reshape(4, 4), it, tr[:int(ex[0])]


def gicp_linearize(src, src_cov, tgt, tgt_cov, T, textbook=False):
    """The GICP linearisation at T: (corr (ns,), H (6,6), b (6,), error) -- the spec's arithmetic (textbook=False)
    or the independent long-double 4x4 restatement (textbook=True), both on the spec's correspondences."""
    src = _c(src, np.float32).reshape(-1, 3)
    tgt = _c(tgt, np.float32).reshape(-1, 3)
    corr = np.zeros(max(len(src), 1), np.int32)
    sys = np.zeros(28, np.float64)
    _gicp_lib().orc_gicp_linearize(src.reshape(-1), _c(src_cov, np.float64).reshape(-1), len(src), tgt.reshape(-1),
                                   _c(tgt_cov, np.float64).reshape(-1), len(tgt), _c(T, np.float64).reshape(-1),
                                   int(bool(textbook)), corr, sys)
    H = np.zeros((6, 6))
    iu = np.triu_indices(6)
    H[iu] = sys[:21]
    H = H + np.triu(H, 1).T
    return corr[:len(src)], H, sys[21:27].copy(), float(sys[27])


def gicp_se3_exp(a):
    out = np.zeros(16, np.float64)
    _gicp_lib().orc_gicp_se3_exp(_c(a, np.float64).reshape(-1), out)
    return out.reshape(4, 4)


def gicp_lm_solve(H, b, lam):
    iu = np.triu_indices(6)
    sys = np.concatenate([np.asarray(H, np.float64)[iu], np.asarray(b, np.float64), [0.0]])
    d = np.zeros(6, np.float64)
    _gicp_lib().orc_gicp_lm_solve(sys, float(lam), d)
    return d


def gicp_lm_solve_sys(sys, lam):
    """The damped solve of a raw 28-term system (upper H row-major, b, error): pcore_gicp_math.h lm_solve_schur, the
    kernels' solve."""
    sys = np.ascontiguousarray(sys, np.float64).reshape(28)
    d = np.zeros(6, np.float64)
    _gicp_lib().orc_gicp_lm_solve(sys, float(lam), d)
    return d


def gicp_lm_solve_ldlt_sys(sys, lam):
    """The same system solved by Eigen's pivoted LDLT (fast_gicp's solve; a test reference)."""
    sys = np.ascontiguousarray(sys, np.float64).reshape(28)
    d = np.zeros(6, np.float64)
    _gicp_lib().orc_gicp_lm_solve_ldlt(sys, float(lam), d)
    return d


def sin_d(x):
    return _gicp_lib().orc_sin_d(float(x))


def cos_d(x):
    return _gicp_lib().orc_cos_d(float(x))


def cube_rn(u):
    return _gicp_lib().orc_cube_rn(float(u))


def lm_gain(rho):
    return _gicp_lib().orc_lm_gain(float(rho))


def gicp_nn(q, tgt):
    q = _c(q, np.float32).reshape(-1, 3)
    tgt = _c(tgt, np.float32).reshape(-1, 3)
    out = np.zeros(max(len(q), 1), np.int32)
    _gicp_lib().orc_gicp_nn(q.reshape(-1), len(q), tgt.reshape(-1), len(tgt), out)
    return out[:len(q)]


def concat_pose(T, pose):
    out = np.zeros(16, np.float32)
    _gicp_lib().orc_concat_pose(_c(T, np.float64).reshape(-1), _c(pose, np.float32).reshape(-1), out)
    return out


def evaluate_icp(tris, tris_model_count, poses, pose_model, pose_label, width, height, proj, src_depth, src_mask,
                 occlusion_threshold, stride, cx, cy, fx, fy, depth_factor, o_xyz, o_cov, label_start, label_end,
                 pose_obs_total, cost_type, calc_obs, sensor_resolution, k=GICP_K, max_iter=GICP_MAX_ITER,
                 rot_eps=GICP_ROT_EPS, trans_eps=GICP_TRANS_EPS, nthreads=0, cycle_window=GICP_CYCLE_WINDOW):
    """do_icp flow; returns (adjusted poses (N,16), iterations (N,), rc, oc, diff)."""
    tris = _c(tris, np.float32).reshape(-1)
    poses = _c(poses, np.float32).reshape(-1)
    n = poses.size // 16
    o_xyz = _c(o_xyz, np.float32).reshape(-1)
    o_cov = _c(o_cov, np.float64).reshape(-1)
    adj = np.zeros((n, 16), np.float32)
    iters = np.zeros(n, np.int32)
    rc = np.zeros(n, np.float32)
    oc = np.zeros(n, np.float32)
    df = np.zeros(n, np.float32)
    nl = 0 if label_start is None else len(label_start)
    _gicp_lib().orc_evaluate_icp(
        tris, tris.size // 9, _c(tris_model_count, np.int32), len(tris_model_count), poses, _c(pose_model, np.int32),
        _c(pose_label, np.int32), n, width, height, _c(proj, np.float32), _c(src_depth, np.int32).reshape(-1),
        None if src_mask is None else _c(src_mask, np.uint8).reshape(-1), float(occlusion_threshold), stride, cx, cy,
        fx, fy, depth_factor, o_xyz if o_xyz.size else np.zeros(3, np.float32),
        o_cov if o_cov.size else np.zeros(6, np.float64), o_xyz.size // 3, _c(label_start, np.int32),
        _c(label_end, np.int32), nl, _c(pose_obs_total, np.float32), cost_type, int(calc_obs), sensor_resolution, k,
        max_iter, rot_eps, trans_eps, int(cycle_window), adj.reshape(-1), iters, rc, oc, df, nthreads)
    return adj, iters, rc, oc, df


def pose_distances(pts, T_gt, T_est, chunk=2048):
    """ADD / ADD-S per pose pair, float64 brute force (pose_error.py:72-108; fat_pose_image.py:2116-2136):
    ADD = mean_i |G p_i - E p_i|, ADD-S = mean_i min_j |G p_i - E p_j|."""
    P = np.asarray(pts, np.float64).reshape(-1, 3)
    G = np.asarray(T_gt, np.float64).reshape(-1, 4, 4)
    E = np.asarray(T_est, np.float64).reshape(-1, 4, 4)
    add = np.zeros(len(G))
    adds = np.zeros(len(G))
    for m in range(len(G)):
        a = P @ G[m, :3, :3].T + G[m, :3, 3]
        b = P @ E[m, :3, :3].T + E[m, :3, 3]
        add[m] = np.linalg.norm(a - b, axis=1).mean()
        best = np.empty(len(a))
        for c0 in range(0, len(a), chunk):
            d = ((a[c0:c0 + chunk, None, :] - b[None, :, :]) ** 2).sum(-1)
            best[c0:c0 + chunk] = np.sqrt(d.min(1))
        adds[m] = best.mean()
    return add, adds


def _colour_lib():
    L = lib()
    if not getattr(L, "_colour_ready", False):
        f = ctypes.c_float
        L.orc_rgb2lab.argtypes = [_u8p, _f32p]
        L.orc_colour_distance.argtypes = [_f32p, _f32p]
        L.orc_colour_distance.restype = ctypes.c_double
        for n in ("orc_sin_f", "orc_cos_f", "orc_exp_f"):
            getattr(L, n).argtypes = [f]
            getattr(L, n).restype = f
        L.orc_atan2_f.argtypes = [f, f]
        L.orc_atan2_f.restype = f
        L.orc_evaluate_colour.argtypes = [
            _f32p, ctypes.c_int, _u8p, _i32p, ctypes.c_int, _f32p, _i32p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
            _f32p, _i32p, f, ctypes.c_int, f, f, f, f, f, _f32p, _u8p, ctypes.c_int, _f32p, ctypes.c_int, f, f,
            _f32p, _f32p, _f32p, ctypes.c_int]
        L._colour_ready = True
    return L


def rgb2lab(rgb):
    """(3,) uint8 -> (3,) float32 Lab with the reference cost's channel order."""
    out = np.zeros(3, np.float32)
    _colour_lib().orc_rgb2lab(_c(rgb, np.uint8).reshape(3), out)
    return out


def colour_distance(lab1, lab2) -> float:
    return _colour_lib().orc_colour_distance(_c(lab1, np.float32).reshape(3), _c(lab2, np.float32).reshape(3))


def colour_math(name, *args) -> float:
    return getattr(_colour_lib(), "orc_" + name)(*[float(a) for a in args])


def evaluate_colour(tris, tri_rgb, tris_model_count, poses, pose_model, width, height, proj, src_depth,
                    occlusion_threshold, stride, cx, cy, fx, fy, depth_factor, o_xyz, o_rgb, pose_obs_total,
                    calc_obs=True, sensor_resolution=0.01, colour_thr=15.0, nthreads=0):
    """Cost type 1 (3-DoF RGB-D) for every pose -> (rc, oc, diff)."""
    tris = _c(tris, np.float32).reshape(-1)
    poses = _c(poses, np.float32).reshape(-1)
    n = poses.size // 16
    o_xyz = _c(o_xyz, np.float32).reshape(-1)
    rc = np.zeros(n, np.float32)
    oc = np.zeros(n, np.float32)
    df = np.zeros(n, np.float32)
    _colour_lib().orc_evaluate_colour(
        tris, tris.size // 9, _c(tri_rgb, np.uint8).reshape(-1), _c(tris_model_count, np.int32),
        len(tris_model_count), poses, _c(pose_model, np.int32), n, width, height, _c(proj, np.float32),
        _c(src_depth, np.int32).reshape(-1), float(occlusion_threshold), stride, cx, cy, fx, fy, depth_factor,
        o_xyz if o_xyz.size else np.zeros(3, np.float32),
        _c(o_rgb, np.uint8).reshape(-1) if o_xyz.size else np.zeros(3, np.uint8), o_xyz.size // 3,
        _c(pose_obs_total, np.float32), int(calc_obs), sensor_resolution, colour_thr, rc, oc, df, nthreads)
    return rc, oc, df


# ---- a14: the reference's CPU/OMP path (ref_cpu_path.cpp) -------------------------------------------
# ICPConvergenceCriteria defaults (cuda_icp/include/cuda_icp/icp.h:39-51) and Scene_projective's
# max_dist_diff default (depth_scene.h:11)
REF_ICP_REL_FITNESS = 1e-5
REF_ICP_REL_RMSE = 1e-5
REF_ICP_MAX_ITER = 30
REF_SCENE_MAX_DIST_DIFF = 0.1


def _ref_lib():
    L = lib()
    if not getattr(L, "_ref_ready", False):
        c_int, f = ctypes.c_int, ctypes.c_float
        L.orc_ref_render_cpu.argtypes = [_f32p, c_int, _f32p, c_int, c_int, c_int, _f32p, _i32p, c_int]
        L.orc_ref_depth2cloud.restype = c_int
        L.orc_ref_depth2cloud.argtypes = [_i32p, c_int, c_int, f, f, f, f, _f32p, c_int]
        L.orc_ref_scene.argtypes = [_i32p, c_int, c_int, f, f, f, f, _f32p, _f32p]
        L.orc_ref_icp.restype = c_int
        L.orc_ref_icp.argtypes = [_f32p, c_int, _f32p, _f32p, c_int, c_int, f, f, f, f, f, f, f, c_int, _f32p,
                                  ctypes.POINTER(f), ctypes.POINTER(f)]
        L.orc_ref_cpu_pipeline.argtypes = [_f32p, c_int, _f32p, c_int, c_int, c_int, _f32p, f, f, f, f, _i32p, f, f,
                                           f, c_int, _f32p, _f32p, _f32p, _opt(_i32p), _opt(_i32p), c_int]
        L.orc_ref_solver666.argtypes = [_f32p, _f32p, _f32p]
        L._ref_ready = True
    return L


def ref_render_cpu(tris, poses, width, height, proj, nthreads=0):
    """render_cpu (renderer.cpp:291-330): (N, H, W) int32 cm, no source occlusion."""
    tris = _c(tris, np.float32).reshape(-1)
    poses = _c(poses, np.float32).reshape(-1)
    n = poses.size // 16
    out = np.zeros((n, height, width), np.int32)
    _ref_lib().orc_ref_render_cpu(tris, tris.size // 9, poses, n, width, height, _c(proj, np.float32), out, nthreads)
    return out


def ref_depth2cloud(depth, fx, fy, cx, cy):
    """depth2cloud_cpu at stride 1 (icp.cpp:64-108): (P, 3) float32 metres, row-major order."""
    d = _c(depth, np.int32)
    h, w = d.shape
    out = np.zeros((h * w, 3), np.float32)
    n = _ref_lib().orc_ref_depth2cloud(d.reshape(-1), w, h, fx, fy, cx, cy, out.reshape(-1), h * w)
    return out[:n]


def ref_scene(depth, fx, fy, cx, cy):
    """Scene_projective buffers: (H, W, 3) points (dep2pcd) and (H, W, 3) get_normal normals."""
    d = _c(depth, np.int32)
    h, w = d.shape
    pcd = np.zeros((h, w, 3), np.float32)
    nrm = np.zeros((h, w, 3), np.float32)
    _ref_lib().orc_ref_scene(d.reshape(-1), w, h, fx, fy, cx, cy, pcd.reshape(-1), nrm.reshape(-1))
    return pcd, nrm


def ref_icp(model_xyz, scene_pcd, scene_normal, fx, fy, cx, cy, max_dist_diff=REF_SCENE_MAX_DIST_DIFF,
            rel_fitness=REF_ICP_REL_FITNESS, rel_rmse=REF_ICP_REL_RMSE, max_iter=REF_ICP_MAX_ITER):
    """ICP_Point2Plane_cpu (icp.cpp:116-179) -> (T (4,4) f32, fitness, rmse, iteration, moved cloud)."""
    pts = np.array(model_xyz, np.float32, copy=True).reshape(-1)
    h, w = scene_pcd.shape[:2]
    T = np.zeros(16, np.float32)
    fit, rmse = ctypes.c_float(0), ctypes.c_float(0)
    it = _ref_lib().orc_ref_icp(pts, pts.size // 3, _c(scene_pcd, np.float32).reshape(-1),
                                _c(scene_normal, np.float32).reshape(-1), w, h, fx, fy, cx, cy, max_dist_diff,
                                rel_fitness, rel_rmse, max_iter, T, ctypes.byref(fit), ctypes.byref(rmse))
    return T.reshape(4, 4), fit.value, rmse.value, it, pts.reshape(-1, 3)


def ref_solver666(A, b):
    """eigen_slover_666 (icp.cpp:29-36): LDLT solve in double, ZYX Euler + translation -> (4,4) float32."""
    out = np.zeros(16, np.float32)
    _ref_lib().orc_ref_solver666(np.ascontiguousarray(np.asarray(A, np.float32).T).reshape(-1),
                                 _c(b, np.float32).reshape(6), out)
    return out.reshape(4, 4)


def ref_cpu_pipeline(tris, poses, width, height, proj, fx, fy, cx, cy, scene_depth_cm,
                     max_dist_diff=REF_SCENE_MAX_DIST_DIFF, rel_fitness=REF_ICP_REL_FITNESS,
                     rel_rmse=REF_ICP_REL_RMSE, max_iter=REF_ICP_MAX_ITER, nthreads=0):
    """a14 per pose: render_cpu -> depth2cloud_cpu -> ICP_Point2Plane_cpu vs the projective scene.
    Returns (T (N,4,4), fitness (N,), rmse (N,), iterations (N,), rendered points (N,))."""
    tris = _c(tris, np.float32).reshape(-1)
    poses = _c(poses, np.float32).reshape(-1)
    n = poses.size // 16
    T = np.zeros((n, 16), np.float32)
    fit = np.zeros(n, np.float32)
    rmse = np.zeros(n, np.float32)
    its = np.zeros(n, np.int32)
    pts = np.zeros(n, np.int32)
    _ref_lib().orc_ref_cpu_pipeline(tris, tris.size // 9, poses, n, width, height, _c(proj, np.float32), fx, fy, cx,
                                    cy, _c(scene_depth_cm, np.int32).reshape(-1), max_dist_diff, rel_fitness,
                                    rel_rmse, max_iter, T.reshape(-1), fit, rmse, its, pts, nthreads)
    return T.reshape(n, 4, 4), fit, rmse, its, pts
