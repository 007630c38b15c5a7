"""Pose proposals of the YCB harness: the candidate list that the search scores.

The reference builds it in Python and hands it to the C++ search through `poses.txt`:

- viewpoints on a Fibonacci sphere (sphere_fibonacci_grid_points.py:7-100), half or whole per object;
- each viewpoint turned into xyz Euler angles, with per-object in-plane (yaw) samples
  (FATImage.get_rotation_samples, fat_pose_image.py:1171-1281; cart2sphere from dipy, sphere2euler from
  convert_fat_coco.py:348-352; euler2quat 'sxyz' from lib/pair_matching/RT_transform.py:527-592);
- a depth sweep along the ray through the object's mask centroid, from the mask's min to max depth in
  steps of 2 cm (1 cm for scissors), every rotation at every depth (fat_pose_image.py:1571-1663, with
  get_world_point at 340-350);
- rows `x y z qx qy qz qw` in metres, rounded to 4 decimals, written with np.savetxt
  (fat_pose_image.py:760-775) and parsed by GenerateSuccessorStates (search_env.cpp:7098-7130).

Everything here is host-side list building (O(viewpoints x depths)); the scoring of the list is the
GPU hot path.
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence, Tuple

import numpy as np

# Per-object symmetry of the proposal sphere: [half (0) / whole (1) sphere, yaw mode]
# (name_sym_dict, fat_pose_image.py:1174-1216; the commented-out alternatives there are not used).
SYMMETRY: Dict[str, Tuple[int, int]] = {
    "002_master_chef_can": (0, 0),
    "003_cracker_box": (0, 0),
    "004_sugar_box": (0, 3),
    "005_tomato_soup_can": (0, 0),
    "006_mustard_bottle": (0, 0),
    "007_tuna_fish_can": (0, 0),
    "008_pudding_box": (0, 1),
    "009_gelatin_box": (0, 0),
    "010_potted_meat_can": (0, 0),
    "011_banana": (1, 0),
    "019_pitcher_base": (0, 0),
    "021_bleach_cleanser": (0, 0),
    "024_bowl": (1, 0),
    "025_mug": (0, 1),
    "035_power_drill": (0, 7),
    "036_wood_block": (0, 0),
    "037_scissors": (0, 2),
    "040_large_marker": (1, 0),
    "052_extra_large_clamp": (0, 7),
    "051_large_clamp": (0, 7),
    "061_foam_brick": (0, 0),
}
SYMMETRY.update({f"color_block_{i}": (0, 8) for i in range(13)})


def sphere_fibonacci_grid_points(ng: int) -> np.ndarray:
    """Whole-sphere Fibonacci lattice (sphere_fibonacci_grid_points.py:7-54): ng points (x, y, z)."""
    return _fibonacci(ng, ng)


def sphere_fibonacci_grid_points_with_sym_metric(ng: int, half_whole: int) -> np.ndarray:
    """sphere_fibonacci_grid_points.py:56-100: whole sphere (half_whole == 1, ng points) or the first
    round(ng / 2) points of the same lattice (half_whole == 0, the y < 0 half)."""
    return _fibonacci(ng, ng if half_whole == 1 else round(ng / 2))


def _fibonacci(samples: int, count: int) -> np.ndarray:
    rnd = 1.0
    offset = 2.0 / samples
    increment = math.pi * (3.0 - math.sqrt(5.0))
    pts = []
    for i in range(count):
        y = ((i * offset) - 1) + (offset / 2)
        r = math.sqrt(1 - pow(y, 2))
        phi = ((i + rnd) % samples) * increment
        pts.append([math.cos(phi) * r, y, math.sin(phi) * r])
    return np.array(pts)


def cart2sphere(x: float, y: float, z: float) -> Tuple[float, float, float]:
    """dipy.core.geometry.cart2sphere (dipy is not vendored in the reference; its published definition):
    r = |p|, theta = arccos(z / r) (0 at r = 0), phi = arctan2(y, x)."""
    r = math.sqrt(x * x + y * y + z * z)
    theta = math.acos(z / r) if r > 0 else 0.0
    return r, theta, math.atan2(y, x)


def sphere2euler(theta: float, phi: float) -> Tuple[float, float]:
    """convert_fat_coco.py:348-352."""
    return math.pi / 2 - theta, phi


def euler2quat(ai: float, aj: float, ak: float) -> np.ndarray:
    """Quaternion (w, x, y, z) of static-frame xyz Euler angles ('sxyz'), sign-normalised to w >= 0
    (RT_transform.euler2quat, RT_transform.py:527-592, for axes 'sxyz': first axis x, no parity, no
    repetition, static frame)."""
    ai, aj, ak = ai / 2.0, aj / 2.0, ak / 2.0
    ci, si = math.cos(ai), math.sin(ai)
    cj, sj = math.cos(aj), math.sin(aj)
    ck, sk = math.cos(ak), math.sin(ak)
    cc, cs, sc, ss = ci * ck, ci * sk, si * ck, si * sk
    q = np.array([cj * cc + sj * ss, cj * sc - sj * cs, cj * ss + sj * cc, cj * cs - sj * sc])
    if q[0] < 0:
        q *= -1
    return q


def quat_wxyz_to_xyzw(q: Sequence[float]) -> List[float]:
    """get_xyzw_quaternion (convert_fat_coco.py:330-331)."""
    q = list(q)
    return q[1:4] + [q[0]]


def _yaw_range(stop: float, step: float) -> np.ndarray:
    return np.arange(0, stop, step)


def rotation_samples(label: str, num_samples: int) -> List[List[float]]:
    """FATImage.get_rotation_samples (fat_pose_image.py:1171-1281): xyz Euler triples per viewpoint.

    Yaw modes (second entry of SYMMETRY): 0 one sample; 1 yaw in [0, pi) step pi/2; 2 [0, pi) step pi/4;
    3 yaw 0 and 2pi/3; 4 upright (pi + theta about y); 5 flipped; 6 yaw 0, pi/3, 2pi/3; 7 [0, 2pi) step
    pi/2; 8 about the first axis in [0, pi) step pi/3.  Unknown labels raise KeyError, as the reference."""
    half_whole, mode = SYMMETRY[label]
    out: List[List[float]] = []
    for vx, vy, vz in sphere_fibonacci_grid_points_with_sym_metric(num_samples, half_whole):
        _, theta, phi = cart2sphere(vx, vy, vz)
        theta, phi = sphere2euler(theta, phi)
        if mode == 0:
            out.append([-phi, theta, 0])
        elif mode == 1:
            out += [[-phi, yaw, theta] for yaw in _yaw_range(math.pi, math.pi / 2)]
        elif mode == 2:
            out += [[-phi, yaw, theta] for yaw in _yaw_range(math.pi, math.pi / 4)]
        elif mode == 3:
            out += [[-phi, 0, theta], [-phi, 2 * math.pi / 3, theta]]
        elif mode == 4:
            out.append([-phi, math.pi + theta, 0])
        elif mode == 5:
            out.append([phi, theta, math.pi])
        elif mode == 6:
            out += [[-phi, 0, theta], [-phi, math.pi / 3, theta], [-phi, 2 * math.pi / 3, theta]]
        elif mode == 7:
            out += [[-phi, yaw, theta] for yaw in _yaw_range(2 * math.pi, math.pi / 2)]
        elif mode == 8:
            out += [[yaw, -phi, theta] for yaw in _yaw_range(math.pi, math.pi / 3)]
    return out


def rotation_quaternions(label: str, num_samples: int) -> List[List[float]]:
    """The object_rotation_list of fat_pose_image.py:1591-1596: xyzw quaternions of rotation_samples."""
    return [quat_wxyz_to_xyzw(euler2quat(a[0], a[1], a[2]).tolist()) for a in rotation_samples(label, num_samples)]


def get_world_point(K: np.ndarray, point: Sequence[float]) -> np.ndarray:
    """FATImage.get_world_point (fat_pose_image.py:340-350): pixel (u, v) at depth z -> camera frame."""
    fx_r = 1.0 / K[0, 0]
    fy_r = 1.0 / K[1, 1]
    out = np.zeros(3)
    out[2] = point[2]
    out[0] = (point[0] - K[0, 2]) * point[2] * fx_r
    out[1] = (point[1] - K[1, 2]) * point[2] * fy_r
    return out


def depth_sweep(object_depth: np.ndarray, depth_factor: float, label: str) -> np.ndarray:
    """Depths of the sweep (fat_pose_image.py:1578-1580, 1628-1631, 1644): min..max of the object's
    masked depth (metres) in steps of 2 cm (1 cm for 037_scissors), max + step exclusive."""
    vals = object_depth[object_depth > 0]
    lo = np.min(vals) / depth_factor
    hi = np.max(vals) / depth_factor
    res = 0.01 if label == "037_scissors" else 0.02
    return np.arange(lo, hi + res, res)


def object_proposals(label: str, centroid_2d: Sequence[float], object_depth: np.ndarray, depth_factor: float,
                     K: np.ndarray, num_samples: int) -> np.ndarray:
    """Rows (x, y, z, qx, qy, qz, qw), metres, for one detected object: every rotation at every depth of
    the sweep along the centroid ray, depth-major (fat_pose_image.py:1644-1654).  io.write_poses_txt
    rounds them to 4 decimals as the reference does when it writes poses.txt (760-775)."""
    quats = rotation_quaternions(label, num_samples)
    rows = []
    for depth in depth_sweep(object_depth, depth_factor, label):
        c = get_world_point(K, list(centroid_2d) + [depth])
        for q in quats:
            rows.append(list(c) + list(q))
    return np.asarray(rows, np.float64).reshape(-1, 7)
