"""Synthetic inputs for tests and benchmarks (no YCB-Video / PoseCNN data offline).

- YCB proxies: boxes / cylinders with YCB nominal dimensions, every face tessellated.
  The 003_cracker_box proxy (0.060 x 0.158 x 0.210 m, 32 x 32 quads per face) has 12,288 triangles.
- Scan-like irregular meshes (scan_blob closed, scan_shell open; ~20-24 k triangles, varied triangle sizes and
  valence, slivers, shuffled face order), as the reference's assimp meshes of real scans are (model.cpp:16-49).
- Camera: the reference's 640x480 intrinsics (sbpl_perception/config/camera_config.yaml:2-7) and the
  1280x720 variant of C5.
- Scenes: GT poses rendered with a caller-supplied depth renderer (the GPU RENDER stage on the box, the
  CPU oracle in CPU tests), 16-bit depth at depth_factor 10000 with N(0, 2 mm) noise, a background
  plane (label 0) and a label mask.
- Candidate poses: fibonacci viewpoints x in-plane yaw x (depth sweep + jitter) around the GT centroid,
  in the spirit of fat_pose_image.py:1456-1663.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from .model import Model, ModelBank, compute_proj, init_from_eigen_batch

SEED = 20250112

CAM_640 = dict(width=640, height=480, fx=576.09757860, fy=576.09757860, cx=321.06398107, cy=242.97676897)
CAM_1280 = dict(width=1280, height=720, fx=1152.195, fy=1152.195, cx=640.0, cy=360.0)

# (kind, dims) -- box: (x, y, z) extents in metres; cyl: (diameter, height)
YCB_PROXIES = {
    "002_master_chef_can": ("cyl", (0.102, 0.139)),
    "003_cracker_box": ("box", (0.060, 0.158, 0.210)),
    "004_sugar_box": ("box", (0.038, 0.089, 0.175)),
    "005_tomato_soup_can": ("cyl", (0.066, 0.101)),
    "006_mustard_bottle": ("box", (0.050, 0.095, 0.190)),
    "007_tuna_fish_can": ("cyl", (0.085, 0.033)),
    "008_pudding_box": ("box", (0.035, 0.110, 0.089)),
    "009_gelatin_box": ("box", (0.028, 0.085, 0.073)),
    "010_potted_meat_can": ("box", (0.050, 0.097, 0.082)),
    "011_banana": ("box", (0.036, 0.190, 0.036)),
    "019_pitcher_base": ("cyl", (0.108, 0.235)),
    "021_bleach_cleanser": ("box", (0.065, 0.098, 0.250)),
    "024_bowl": ("cyl", (0.159, 0.053)),
    "025_mug": ("cyl", (0.080, 0.082)),
    "035_power_drill": ("box", (0.035, 0.184, 0.187)),
    "036_wood_block": ("box", (0.085, 0.085, 0.200)),
    "037_scissors": ("box", (0.014, 0.087, 0.200)),
    "040_large_marker": ("cyl", (0.018, 0.121)),
    "051_large_clamp": ("box", (0.030, 0.120, 0.170)),
    "052_extra_large_clamp": ("box", (0.030, 0.165, 0.213)),
    "061_foam_brick": ("box", (0.050, 0.075, 0.050)),
}


def box_mesh(dims: Sequence[float], k: int = 32) -> np.ndarray:
    """Axis-aligned box centred at the origin, each face a k x k quad grid (2 triangles per quad),
    outward winding.  Returns (12 k^2, 9) float32."""
    hx, hy, hz = (0.5 * float(d) for d in dims)
    tris = []
    u = np.linspace(-1.0, 1.0, k + 1)
    # each face: fixed axis, sign, the two in-plane axes
    for axis, sign in ((0, 1), (0, -1), (1, 1), (1, -1), (2, 1), (2, -1)):
        a1, a2 = [a for a in range(3) if a != axis]
        if sign < 0:
            a1, a2 = a2, a1
        h = (hx, hy, hz)
        grid = np.zeros((k + 1, k + 1, 3))
        grid[..., axis] = sign * h[axis]
        grid[..., a1] = u[:, None] * h[a1]
        grid[..., a2] = u[None, :] * h[a2]
        for i in range(k):
            for j in range(k):
                p00, p10, p01, p11 = grid[i, j], grid[i + 1, j], grid[i, j + 1], grid[i + 1, j + 1]
                tris.append(np.concatenate([p00, p10, p11]))
                tris.append(np.concatenate([p00, p11, p01]))
    return np.asarray(tris, dtype=np.float32)


def cylinder_mesh(diameter: float, height: float, segments: int = 64, rings: int = 24, cap_rings: int = 8) -> np.ndarray:
    """Closed cylinder along z, centred at the origin."""
    r, hz = 0.5 * float(diameter), 0.5 * float(height)
    th = np.linspace(0.0, 2 * np.pi, segments + 1)
    zs = np.linspace(-hz, hz, rings + 1)
    tris = []
    for i in range(rings):
        for j in range(segments):
            p = lambda a, z: np.array([r * np.cos(th[a]), r * np.sin(th[a]), z])
            p00, p10, p01, p11 = p(j, zs[i]), p(j + 1, zs[i]), p(j, zs[i + 1]), p(j + 1, zs[i + 1])
            tris.append(np.concatenate([p00, p10, p11]))
            tris.append(np.concatenate([p00, p11, p01]))
    rr = np.linspace(0.0, r, cap_rings + 1)
    for zc, sgn in ((hz, 1), (-hz, -1)):
        for i in range(cap_rings):
            for j in range(segments):
                q = lambda ri, a: np.array([rr[ri] * np.cos(th[a]), rr[ri] * np.sin(th[a]), zc])
                q00, q10, q01, q11 = q(i, j), q(i, j + 1), q(i + 1, j), q(i + 1, j + 1)
                if i == 0:
                    t = [np.concatenate([q00, q01, q11])]
                else:
                    t = [np.concatenate([q00, q01, q11]), np.concatenate([q00, q11, q10])]
                if sgn < 0:
                    t = [np.concatenate([x[0:3], x[6:9], x[3:6]]) for x in t]
                tris.extend(t)
    return np.asarray(tris, dtype=np.float32)


def icosphere(level: int):
    """Unit icosphere: (vertices (V, 3) float64, faces (F, 3) int64, outward winding), F = 20 * 4^level."""
    t = (1.0 + 5 ** 0.5) / 2.0
    V = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
         (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    F = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2), (10, 7, 6),
         (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11), (6, 2, 10),
         (8, 6, 7), (9, 8, 1)]
    V = np.asarray(V, np.float64)
    V /= np.linalg.norm(V, axis=1, keepdims=True)
    F = np.asarray(F, np.int64)
    for _ in range(level):
        e = np.concatenate([F[:, [0, 1]], F[:, [1, 2]], F[:, [2, 0]]])
        key = np.sort(e, axis=1)
        uniq, inv = np.unique(key, axis=0, return_inverse=True)
        mid = V[uniq[:, 0]] + V[uniq[:, 1]]
        mid /= np.linalg.norm(mid, axis=1, keepdims=True)
        m = inv.reshape(3, -1).T + len(V)  # midpoints of edges 01, 12, 20
        V = np.concatenate([V, mid])
        a, b, c = F[:, 0], F[:, 1], F[:, 2]
        ab, bc, ca = m[:, 0], m[:, 1], m[:, 2]
        F = np.concatenate([np.stack([a, ab, ca], 1), np.stack([b, bc, ab], 1), np.stack([c, ca, bc], 1),
                            np.stack([ab, bc, ca], 1)])
    return V, F


def scan_mesh(semi_axes: Sequence[float], level: int = 5, open_below: Optional[float] = None, split_frac: float = 0.15,
              seed: int = 0) -> np.ndarray:
    """A scan-like irregular mesh: an icosphere whose vertex density is warped towards one
    side (triangle areas vary ~10x, elongated triangles), displaced by low-frequency bumps and per-vertex noise,
    scaled to an ellipsoid; a fraction of the triangles split at a random point of their longest edge (slivers,
    T-junctions, uneven valence); optionally cut open (faces whose centroid lies below `open_below` on the warped
    z axis are dropped: a partial scan); face order shuffled and each face's vertex order rotated (winding kept).
    Returns (T, 9) float32."""
    rng = np.random.default_rng(seed)
    V, F = icosphere(level)
    d = np.array([0.3, -0.2, 0.93])
    d /= np.linalg.norm(d)
    V = V + 0.55 * d
    V /= np.linalg.norm(V, axis=1, keepdims=True)
    r = np.ones(len(V))
    for _ in range(6):  # low-frequency bumps
        u = rng.normal(size=3)
        u /= np.linalg.norm(u)
        r += 0.05 * np.sin(rng.uniform(2.0, 5.0) * (V @ u) + rng.uniform(0, 2 * np.pi))
    r += rng.normal(0.0, 0.006, len(V))  # sensor-like vertex noise
    V = V * r[:, None] * np.asarray(semi_axes, np.float64)[None, :]
    keep = np.ones(len(F), bool)
    if open_below is not None:
        cz = V[F].mean(1) @ (d * np.asarray(semi_axes)) / np.linalg.norm(d * np.asarray(semi_axes))
        keep = cz > open_below * float(np.max(semi_axes))
    F = F[keep]
    T = V[F]  # (F, 3, 3)
    ns = int(split_frac * len(T))
    sel = rng.choice(len(T), ns, replace=False)
    tris = [np.delete(T, sel, axis=0)]
    for t in T[sel]:
        el = [np.linalg.norm(t[(i + 1) % 3] - t[i]) for i in range(3)]
        i = int(np.argmax(el))
        a, b, c = t[i], t[(i + 1) % 3], t[(i + 2) % 3]
        p = a + rng.uniform(0.1, 0.9) * (b - a)
        tris.append(np.stack([np.stack([a, p, c]), np.stack([p, b, c])]))
    T = np.concatenate(tris)
    T = T[rng.permutation(len(T))]
    rot = rng.integers(0, 3, len(T))
    idx = (np.arange(3)[None, :] + rot[:, None]) % 3
    T = np.take_along_axis(T, idx[:, :, None], axis=1)
    return T.reshape(-1, 9).astype(np.float32)


# scan-like irregular meshes: (semi-axes in metres, icosphere level, open_below, seed)
SCAN_MESHES = {
    "scan_blob": ((0.045, 0.075, 0.100), 5, None, 3),    # closed, ~23.5 k triangles
    "scan_shell": ((0.070, 0.060, 0.080), 5, -0.45, 5),  # open partial scan, ~20 k triangles
}


def ycb_proxy(name: str, k: int = 32) -> Model:
    if name in SCAN_MESHES:
        axes, level, open_below, seed = SCAN_MESHES[name]
        return Model(name=name, tris=scan_mesh(axes, level, open_below, seed=seed))
    kind, dims = YCB_PROXIES[name]
    tris = box_mesh(dims, k) if kind == "box" else cylinder_mesh(*dims)
    return Model(name=name, tris=tris)


def model_bank(names: Sequence[str], k: int = 32) -> ModelBank:
    return ModelBank([ycb_proxy(n, k) for n in names])


# ---------------------------------------------------------------------------------------------
# rotations / poses
# ---------------------------------------------------------------------------------------------

def fibonacci_half_sphere(ng: int) -> np.ndarray:
    """sphere_fibonacci_grid_points_with_sym_metric(ng, 0) (sphere_fibonacci_grid_points.py:56-100)."""
    rnd = 1.0
    offset = 2.0 / ng
    increment = np.pi * (3.0 - np.sqrt(5.0))
    pts = []
    for i in range(round(ng / 2)):
        y = ((i * offset) - 1) + (offset / 2)
        r = np.sqrt(1 - y ** 2)
        phi = ((i + rnd) % ng) * increment
        pts.append([np.cos(phi) * r, y, np.sin(phi) * r])
    return np.array(pts)


def _rot_align_z(v: np.ndarray) -> np.ndarray:
    """Rotation taking +z to unit vector v."""
    v = v / np.linalg.norm(v)
    z = np.array([0.0, 0.0, 1.0])
    c = float(np.dot(z, v))
    if c > 1 - 1e-12:
        return np.eye(3)
    if c < -1 + 1e-12:
        return np.diag([1.0, -1.0, -1.0])
    ax = np.cross(z, v)
    s = np.linalg.norm(ax)
    ax = ax / s
    K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    return np.eye(3) + s * K + (1 - c) * (K @ K)


def _rot_z(a: float) -> np.ndarray:
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1.0]])


def rotation_samples(num_viewpoints: int = 80, inplane: int = 8) -> np.ndarray:
    rots = []
    for v in fibonacci_half_sphere(num_viewpoints):
        Ra = _rot_align_z(np.asarray(v))
        for j in range(inplane):
            rots.append(Ra @ _rot_z(2 * np.pi * j / inplane))
    return np.asarray(rots)


def candidate_poses(center: Sequence[float], n: int, rng: np.random.Generator, num_viewpoints: int = 80,
                    inplane: int = 8, depth_step: float = 0.02, depth_span: float = 0.10,
                    jitter: float = 0.05, include: Optional[np.ndarray] = None) -> np.ndarray:
    """n camera-frame 4x4 poses (float64): rotations x (depth sweep along the centroid ray + uniform
    +-jitter), truncated to n.  `include` (4x4) is written at index n // 3 (a GT pose to find)."""
    rots = rotation_samples(num_viewpoints, inplane)
    c = np.asarray(center, dtype=np.float64)
    ray = c / np.linalg.norm(c)
    depths = np.arange(-depth_span, depth_span + 1e-9, depth_step)
    trans = [c + d * ray for d in depths]
    per_rot = int(np.ceil(n / len(rots)))
    while len(trans) < per_rot:
        trans.append(c + rng.uniform(-jitter, jitter, 3))
    out = np.zeros((len(rots) * per_rot, 4, 4))
    k = 0
    for ti in range(per_rot):
        for R in rots:
            out[k, :3, :3] = R
            out[k, :3, 3] = trans[ti]
            out[k, 3, 3] = 1.0
            k += 1
    out = out[:n]
    if include is not None and n > 0:
        out[n // 3] = include
    return out


# ---------------------------------------------------------------------------------------------
# scenes
# ---------------------------------------------------------------------------------------------

@dataclass
class Scene:
    width: int
    height: int
    fx: float
    fy: float
    cx: float
    cy: float
    proj: np.ndarray            # (16,) float32
    bank: ModelBank
    gt_model: List[int]
    gt_poses: np.ndarray        # (K, 4, 4) camera frame, metres
    depth_raw: np.ndarray       # (H, W) int32, sensor units at depth_factor
    mask: np.ndarray            # (H, W) uint8 labels (object k -> k+1, 0 = background)
    depth_factor: float         # raw units per metre (YCB 10000)

    @property
    def src_depth_cm(self) -> np.ndarray:
        """search_env.cpp:2487-2498: input_depth_image_vec[i] /= (depth_factor / 100) on int32."""
        div = np.float32(self.depth_factor) / np.float32(100.0)
        return (self.depth_raw.astype(np.float32) / div).astype(np.int32)


RenderFn = Callable[[np.ndarray, np.ndarray, np.ndarray, np.ndarray, int, int, np.ndarray], np.ndarray]
# render_fn(tris, tris_model_count, poses16 (N,16) f32, pose_model (N,) i32, width, height, proj) -> (N,H,W) int32 cm


def make_scene(names: Sequence[str], gt_poses: np.ndarray, render_fn: RenderFn, cam: dict = CAM_640,
               depth_factor: float = 10000.0, noise_m: float = 0.002, background_m: float = 1.5,
               rng: Optional[np.random.Generator] = None, k: int = 32) -> Scene:
    rng = rng or np.random.default_rng(SEED)
    bank = model_bank(names, k)
    W, H = cam["width"], cam["height"]
    proj = compute_proj(cam["fx"], cam["fy"], cam["cx"], cam["cy"], W, H)
    K = len(names)
    poses16 = init_from_eigen_batch(gt_poses)
    zb = render_fn(bank.tris, bank.tris_model_count, poses16, np.arange(K, dtype=np.int32), W, H, proj)
    depth_cm = np.zeros((H, W), np.int64)
    mask = np.zeros((H, W), np.uint8)
    for obj in range(K):
        z = zb[obj].astype(np.int64)
        closer = (z > 0) & ((depth_cm == 0) | (z < depth_cm))
        depth_cm[closer] = z[closer]
        mask[closer] = obj + 1
    raw = depth_cm.astype(np.float64) * (depth_factor / 100.0)
    bg = mask == 0
    raw[bg] = background_m * depth_factor
    raw = raw + rng.normal(0.0, noise_m * depth_factor, raw.shape)
    raw = np.clip(np.rint(raw), 0, 65535).astype(np.int32)  # 16-bit sensor depth
    return Scene(W, H, cam["fx"], cam["fy"], cam["cx"], cam["cy"], proj, bank, list(range(K)),
                 np.asarray(gt_poses, dtype=np.float64), raw, mask, float(depth_factor))


def default_gt_pose(rng: np.random.Generator, center=(0.03, -0.02, 0.80)) -> np.ndarray:
    T = np.eye(4)
    T[:3, :3] = _rot_align_z(np.array([0.3, -0.4, 1.0])) @ _rot_z(0.7)
    T[:3, 3] = center
    return T


# ---------------------------------------------------------------------------------------------
# 3-DoF table-top scenes (f4)
# ---------------------------------------------------------------------------------------------

CAM_TO_BODY = np.array([[0, 0, 1, 0], [-1, 0, 0, 0], [0, -1, 0, 0], [0, 0, 0, 1]], np.float64)


def tabletop_camera_pose(height: float, pitch: float = 0.7) -> np.ndarray:
    """Camera body pose in the world (x forward, z up) at `height`, pitched down by `pitch` rad."""
    c, s = np.cos(pitch), np.sin(pitch)
    T = np.eye(4)
    T[:3, :3] = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    T[:3, 3] = [0.0, 0.0, height]
    return T


@dataclass
class TabletopScene:
    width: int
    height: int
    fx: float
    fy: float
    cx: float
    cy: float
    proj: np.ndarray
    bank: ModelBank
    camera_pose: np.ndarray      # body pose in the world
    world_poses: np.ndarray      # (K, 4, 4) object model frame -> world
    depth_raw: np.ndarray        # (H, W) int32 at depth_factor
    rgb: np.ndarray              # (H, W, 3) uint8
    depth_factor: float
    table_height: float


def make_tabletop_scene(names: Sequence[str], placements: Sequence[Tuple[float, float, float]],
                        preprocess: Sequence[np.ndarray], render_fn: RenderFn, table_height: float = 0.7,
                        cam: dict = CAM_640, depth_factor: float = 1000.0, noise_m: float = 0.001,
                        rng: Optional[np.random.Generator] = None, k: int = 32,
                        colors: Optional[Sequence[Sequence[int]]] = None) -> TabletopScene:
    """Objects standing on a table plane z = table_height at (x, y, yaw) (world = ContPose * preprocess),
    seen by a camera 0.6 m above the table looking down the +x axis.  Depth: the table plane by ray
    intersection, objects by `render_fn`; colours: the table grey, object k colours[k]."""
    from .tabletop import yaw_pose_matrix
    rng = rng or np.random.default_rng(SEED)
    bank = model_bank(names, k)
    if colors is not None:
        for m, c in zip(bank.models, colors):
            m.colors = np.tile(np.asarray(c, np.uint8), (m.num_tris, 1))
    W, H = cam["width"], cam["height"]
    proj = compute_proj(cam["fx"], cam["fy"], cam["cx"], cam["cy"], W, H)
    cam_pose = tabletop_camera_pose(table_height + 0.6)
    optical = cam_pose @ CAM_TO_BODY
    world = np.stack([yaw_pose_matrix(x, y, table_height, yaw) @ pre for (x, y, yaw), pre in zip(placements, preprocess)])
    in_cam = np.stack([np.linalg.inv(optical) @ T for T in world])
    zb = render_fn(bank.tris, bank.tris_model_count, init_from_eigen_batch(in_cam), np.arange(len(names), dtype=np.int32),
                   W, H, proj)
    # table plane: ray through pixel (u, v) in the optical frame, intersect with z_world = table_height
    u, v = np.meshgrid(np.arange(W, dtype=np.float64), np.arange(H, dtype=np.float64))
    ray = np.stack([(u - cam["cx"]) / cam["fx"], (v - cam["cy"]) / cam["fy"], np.ones_like(u)], -1)
    dz = ray @ optical[2, :3]
    t = (table_height - optical[2, 3]) / np.where(np.abs(dz) > 1e-9, dz, np.nan)
    table_m = np.where(t > 0, t, 0.0)
    table_m = np.nan_to_num(table_m, nan=0.0)
    depth_m = table_m.copy()
    rgb = np.zeros((H, W, 3), np.uint8)
    rgb[table_m > 0] = (90, 90, 90)
    for obj in range(len(names)):
        z = zb[obj].astype(np.float64) / 100.0
        closer = (z > 0) & ((depth_m == 0) | (z < depth_m))
        depth_m[closer] = z[closer]
        rgb[closer] = bank.models[obj].colors[0]
    raw = depth_m * depth_factor + rng.normal(0.0, noise_m * depth_factor, depth_m.shape) * (depth_m > 0)
    raw = np.clip(np.rint(raw), 0, 65535).astype(np.int32)
    return TabletopScene(W, H, cam["fx"], cam["fy"], cam["cx"], cam["cy"], proj, bank, cam_pose, world, raw, rgb,
                         float(depth_factor), float(table_height))
