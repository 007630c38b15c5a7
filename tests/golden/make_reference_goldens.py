"""Generate golden vectors by importing the reference's own Python modules (THIS container only; the
reference never travels to the GPU box).  Run from the repo root:

    python tests/golden/make_reference_goldens.py

- sphere_fibonacci_grid_points.py (sbpl_perception/src/scripts/tools/fat_dataset/) -> fibonacci.npz
- lib/utils/pose_error.py add / adi on seeded poses and model points -> pose_error.npz
"""
import os
import sys

import numpy as np

REF = "/root/reference/sbpl_perception/src/scripts/tools/fat_dataset"
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    sys.path.insert(0, REF)
    import sphere_fibonacci_grid_points as sfg  # noqa: E402

    np.savez(os.path.join(OUT, "fibonacci.npz"),
             half_80=sfg.sphere_fibonacci_grid_points_with_sym_metric(80, 0),
             whole_80=sfg.sphere_fibonacci_grid_points_with_sym_metric(80, 1),
             half_41=sfg.sphere_fibonacci_grid_points_with_sym_metric(41, 0),
             plain_80=sfg.sphere_fibonacci_grid_points(80))
    sys.path.insert(0, os.path.join(REF, "lib", "utils"))
    try:
        import pose_error  # noqa: E402
    except Exception as e:  # ordinary import error -> no pose_error goldens
        print("pose_error not importable:", e)
        return
    rng = np.random.default_rng(20250112)
    pts = rng.uniform(-0.1, 0.1, (500, 3))
    cases = []
    for i in range(6):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        x, y, z, w = q
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                      [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                      [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
        t = rng.uniform(-0.5, 0.5, (3, 1))
        R2 = R @ np.array([[np.cos(0.1 * i), -np.sin(0.1 * i), 0], [np.sin(0.1 * i), np.cos(0.1 * i), 0], [0, 0, 1]])
        t2 = t + rng.normal(0, 0.01 * i, (3, 1))
        cases.append((R2, t2, R, t, pose_error.add(R2, t2, R, t, pts), pose_error.adi(R2, t2, R, t, pts)))
    np.savez(os.path.join(OUT, "pose_error.npz"), pts=pts,
             R_est=np.stack([c[0] for c in cases]), t_est=np.stack([c[1] for c in cases]),
             R_gt=np.stack([c[2] for c in cases]), t_gt=np.stack([c[3] for c in cases]),
             add=np.array([c[4] for c in cases]), adi=np.array([c[5] for c in cases]))


if __name__ == "__main__":
    main()
