"""Host-side mirror of cuda_renderer's Model types (cuda_renderer/include/cuda_renderer/model.h).

- Triangle soups are (T, 9) float32 arrays (v0, v1, v2), metres; colours (T, 3) uint8 from vertex 0
  (model.cpp:81-97, default 128).
- mat4x4 is a (16,) float32 row-major array a0..d3 (model.h:76-81).  `init_from_eigen(pose, 100)` scales
  the rotation AND translation rows by 100 (model.h:89-107) so vertices render in centimetres;
  `to_eigen(m, 100)` is its inverse (model.h:108-127).
- compute_proj restates renderer.cu:1386-1410 with the same float32 operation order.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Sequence

import numpy as np

f32 = np.float32


def compute_proj(fx: float, fy: float, cx: float, cy: float, width: int, height: int,
                 near: float = 10.0, far: float = 10000.0) -> np.ndarray:
    """renderer.cu:1386-1410 (K(0,1) = 0).  Defaults near=10, far=10000 (renderer.h:87)."""
    fx, fy, cx, cy, near, far = (f32(v) for v in (fx, fy, cx, cy, near, far))
    w, h = f32(width), f32(height)
    two = f32(2.0)
    a0 = two * fx / w
    a1 = -(-two * f32(0.0) / w)
    a2 = -(-two * cx / w + f32(1.0))
    b1 = -(two * fy / h)
    b2 = -(two * cy / h - f32(1.0))
    c2 = -(-(far + near) / (far - near))
    c3 = -two * far * near / (far - near)
    d2 = f32(1.0)
    return np.array([a0, a1, a2, 0, 0, b1, b2, 0, 0, 0, c2, c3, 0, 0, d2, 0], dtype=f32)


def init_from_eigen(pose_in_cam: np.ndarray, scale_factor: int = 100) -> np.ndarray:
    """mat4x4::init_from_eigen (model.h:89-107): double 4x4 -> float32[16], rows 0-2 scaled."""
    p = np.asarray(pose_in_cam, dtype=np.float64).reshape(4, 4)
    out = np.empty(16, dtype=f32)
    out[:12] = (p[:3, :] * scale_factor).astype(f32).reshape(-1)
    out[12:] = p[3, :].astype(f32)
    return out


def init_from_eigen_batch(poses_in_cam: np.ndarray, scale_factor: int = 100) -> np.ndarray:
    p = np.asarray(poses_in_cam, dtype=np.float64).reshape(-1, 4, 4)
    out = np.empty((p.shape[0], 16), dtype=f32)
    out[:, :12] = (p[:, :3, :] * scale_factor).astype(f32).reshape(-1, 12)
    out[:, 12:] = p[:, 3, :].astype(f32)
    return out


def to_eigen(mat: np.ndarray, scale_factor: int = 100) -> np.ndarray:
    """mat4x4::to_eigen (model.h:108-127): float32[16] -> float32 4x4, rows 0-2 divided."""
    m = np.asarray(mat, dtype=f32).reshape(4, 4).copy()
    m[:3, :] = m[:3, :] / f32(scale_factor)
    return m


def quat_xyzw_to_matrix(q: Sequence[float]) -> np.ndarray:
    """Normalised quaternion (x, y, z, w) -> 3x3 rotation (Eigen::Quaterniond::toRotationMatrix)."""
    x, y, z, w = (float(v) for v in q)
    n = np.sqrt((x * x + z * z) + (y * y + w * w))  # Eigen squaredNorm in 2-wide packets (SSE2)
    x, y, z, w = x / n, y / n, z / n, w / n
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ])


def matrix_to_quat_xyzw(R: np.ndarray) -> np.ndarray:
    """3x3 rotation -> quaternion (x, y, z, w) (Eigen::Quaternion(Matrix3) construction)."""
    R = np.asarray(R, dtype=np.float64)
    t = np.trace(R)
    if t > 0:
        s = np.sqrt(t + 1.0) * 2
        w = 0.25 * s
        x = (R[2, 1] - R[1, 2]) / s
        y = (R[0, 2] - R[2, 0]) / s
        z = (R[1, 0] - R[0, 1]) / s
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        w = (R[2, 1] - R[1, 2]) / s
        x = 0.25 * s
        y = (R[0, 1] + R[1, 0]) / s
        z = (R[0, 2] + R[2, 0]) / s
    elif R[1, 1] > R[2, 2]:
        s = np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        w = (R[0, 2] - R[2, 0]) / s
        x = (R[0, 1] + R[1, 0]) / s
        y = 0.25 * s
        z = (R[1, 2] + R[2, 1]) / s
    else:
        s = np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        w = (R[1, 0] - R[0, 1]) / s
        x = (R[0, 2] + R[2, 0]) / s
        y = (R[1, 2] + R[2, 1]) / s
        z = 0.25 * s
    return np.array([x, y, z, w])


def quat_from_matrix_eigen_batch(R: np.ndarray, dtype=np.float32) -> np.ndarray:
    """Eigen::Quaternion<Scalar>(Matrix3) over (N, 3, 3) rotations in Scalar = dtype arithmetic, Eigen's own algorithm
    (Geometry/Quaternion.h, quaternionbase_assign_impl<Other, 3, 3>): with t = trace ((m00 + m11) + m22) > 0,
    t = sqrt(t + 1), w = t / 2, then (x, y, z) = (m21 - m12, m02 - m20, m10 - m01) * (0.5 / t); otherwise i = the
    first largest diagonal entry (m11 > m00, then m22 > m_ii), j = i + 1, k = j + 1 (mod 3),
    t = sqrt(((m_ii - m_jj) - m_kk) + 1), q_i = t / 2 and, scaled by 0.5 / t, w = m_kj - m_jk, q_j = m_ji + m_ij,
    q_k = m_ki + m_ik.  -> (N, 4) (x, y, z, w).  search_env.cpp:2008 builds the adjusted ContPose with
    Quaternionf of the float matrix, hence float32 by default."""
    m = np.asarray(R, dtype=dtype).reshape(-1, 3, 3)
    n = len(m)
    half = dtype(0.5)
    one = dtype(1.0)
    out = np.zeros((n, 4), dtype=dtype)
    tr = (m[:, 0, 0] + m[:, 1, 1]) + m[:, 2, 2]
    pos = tr > 0
    with np.errstate(invalid="ignore", divide="ignore"):
        t = np.sqrt(tr + one)
        s = half / t
        pq = np.stack([(m[:, 2, 1] - m[:, 1, 2]) * s, (m[:, 0, 2] - m[:, 2, 0]) * s, (m[:, 1, 0] - m[:, 0, 1]) * s,
                       half * t], 1)
        i = np.where(m[:, 1, 1] > m[:, 0, 0], 1, 0)
        i = np.where(m[:, 2, 2] > m[np.arange(n), i, i], 2, i)
        j = (i + 1) % 3
        k = (j + 1) % 3
        r = np.arange(n)
        t2 = np.sqrt(((m[r, i, i] - m[r, j, j]) - m[r, k, k]) + one)
        s2 = half / t2
        nq = np.zeros((n, 4), dtype=dtype)
        nq[r, i] = half * t2
        nq[:, 3] = (m[r, k, j] - m[r, j, k]) * s2
        nq[r, j] = (m[r, j, i] + m[r, i, j]) * s2
        nq[r, k] = (m[r, k, i] + m[r, i, k]) * s2
    out[:] = np.where(pos[:, None], pq, nq)
    return out


def so3_log_batch(q_xyzw: np.ndarray, dtype=np.float32) -> np.ndarray:
    """Sophus::SO3<Scalar>::log() of unit quaternions (x, y, z, w) in Scalar = dtype (Sophus so3.hpp logAndTheta,
    epsilon 1e-5 for float, 1e-10 for double): n^2 = (x x + y y) + z z; below epsilon^2 the factor
    2 / w - 2/3 n^2 / (w w^2), else with n = sqrt(n^2) +-pi / n when |w| < epsilon, otherwise 2 atan(n / w) / n;
    the tangent is that factor times (x, y, z).  The reference's Sophus is not vendored (search_env.cpp:2614 is its
    only use on this path): parity unpinned."""
    q = np.asarray(q_xyzw, dtype=dtype).reshape(-1, 4)
    x, y, z, w = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    eps = dtype(1e-5) if dtype == np.float32 else dtype(1e-10)
    two = dtype(2.0)
    sq = (x * x + y * y) + z * z
    with np.errstate(invalid="ignore", divide="ignore"):
        small = two / w - dtype(2.0 / 3.0) * sq / (w * (w * w))
        nn = np.sqrt(sq)
        pi = dtype(np.pi)
        near_pi = np.where(w > 0, pi / nn, -pi / nn)
        general = two * np.arctan(nn / w) / nn
        f = np.where(sq < eps * eps, small, np.where(np.abs(w) < eps, near_pi, general))
    return (f[:, None] * q[:, :3]).astype(dtype)


def matmul_lazy(X: np.ndarray, Y: np.ndarray) -> np.ndarray:
    """Batched 4x4 (or 3x3) products in the operands' own dtype, each entry summed over k in index order as Eigen's
    lazy fixed-size product does without FMA: ((x0 y0 + x1 y1) + x2 y2) + ..."""
    acc = X[..., :, 0, None] * Y[..., None, 0, :]
    for c in range(1, X.shape[-1]):
        acc = acc + X[..., :, c, None] * Y[..., None, c, :]
    return acc


def quat_xyzw_to_matrix_batch(q: np.ndarray) -> np.ndarray:
    """quat_xyzw_to_matrix over (N, 4) quaternions: the same float64 operations per element."""
    q = np.asarray(q, dtype=np.float64).reshape(-1, 4)
    x, y, z, w = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    n = np.sqrt((x * x + z * z) + (y * y + w * w))
    x, y, z, w = x / n, y / n, z / n, w / n
    R = np.empty((len(q), 3, 3))
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - z * w)
    R[:, 0, 2] = 2 * (x * z + y * w)
    R[:, 1, 0] = 2 * (x * y + z * w)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - x * w)
    R[:, 2, 0] = 2 * (x * z - y * w)
    R[:, 2, 1] = 2 * (y * z + x * w)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


def pose_matrix_batch(translations: np.ndarray, quats_xyzw: np.ndarray) -> np.ndarray:
    """pose_matrix over N poses: (N, 4, 4)."""
    t = np.asarray(translations, dtype=np.float64).reshape(-1, 3)
    T = np.zeros((len(t), 4, 4))
    T[:, :3, :3] = quat_xyzw_to_matrix_batch(quats_xyzw)
    T[:, :3, 3] = t
    T[:, 3, 3] = 1.0
    return T


def chain_matmul_batch(A: np.ndarray, T: np.ndarray, B: np.ndarray) -> np.ndarray:
    """A @ (T[i] @ B[i]) for every i -- the grouping of search_env.cpp:1567-1571 (transform = T * preprocess, then
    cam_matrix * transform) -- each product summed over k in index order as Eigen's 4x4 lazy product does without
    FMA, ((a0 b0 + a1 b1) + a2 b2) + a3 b3, independent of BLAS blocking and thread count."""
    def mm(X, Y):
        return (((X[..., :, 0, None] * Y[..., None, 0, :] + X[..., :, 1, None] * Y[..., None, 1, :])
                 + X[..., :, 2, None] * Y[..., None, 2, :]) + X[..., :, 3, None] * Y[..., None, 3, :])
    return mm(np.broadcast_to(A, T.shape), mm(T, B))


def pose_matrix(translation: Sequence[float], quat_xyzw: Sequence[float]) -> np.ndarray:
    """ContPose::GetTransform (object_state.cpp:83-97): Translation3d(x,y,z) * normalised quaternion."""
    T = np.eye(4)
    T[:3, :3] = quat_xyzw_to_matrix(quat_xyzw)
    T[:3, 3] = np.asarray(translation, dtype=np.float64)
    return T


@dataclass
class Model:
    """A triangle mesh as cuda_renderer::Model holds it after LoadModel (model.cpp:16-49)."""
    name: str
    tris: np.ndarray                      # (T, 9) float32, metres
    colors: np.ndarray = None             # (T, 3) uint8

    def __post_init__(self):
        self.tris = np.ascontiguousarray(self.tris, dtype=f32).reshape(-1, 9)
        if self.colors is None:
            self.colors = np.full((self.tris.shape[0], 3), 128, np.uint8)
        self.colors = np.ascontiguousarray(self.colors, dtype=np.uint8).reshape(-1, 3)

    @property
    def num_tris(self) -> int:
        return int(self.tris.shape[0])

    def vertices(self) -> np.ndarray:
        return np.unique(self.tris.reshape(-1, 3), axis=0)


@dataclass
class ModelBank:
    """All models concatenated, as LoadObjFiles builds `tris` + `tris_model_count` (search_env.cpp:253-307)."""
    models: List[Model] = field(default_factory=list)

    @property
    def tris(self) -> np.ndarray:
        return np.concatenate([m.tris for m in self.models], axis=0)

    @property
    def colors(self) -> np.ndarray:
        return np.concatenate([m.colors for m in self.models], axis=0)

    @property
    def tris_model_count(self) -> np.ndarray:
        return np.array([m.num_tris for m in self.models], dtype=np.int32)

    def index(self, name: str) -> int:
        for i, m in enumerate(self.models):
            if m.name == name:
                return i
        raise KeyError(name)
