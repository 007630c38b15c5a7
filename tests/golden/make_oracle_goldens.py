"""Regression fixtures of the CPU oracle on small seeded scenes (inputs + expected outputs).

These do not pin the oracle against the reference (no reference golden exists for the hot path; see
DESIGN.md "Oracle"); they freeze the restatement so that the CPU suite and the GPU parity suite check
against the same committed vectors.  Regenerate only on a deliberate semantic change:

    python tests/golden/make_oracle_goldens.py
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from perception_amd import synthetic as syn  # noqa: E402
from perception_amd.model import compute_proj, init_from_eigen_batch  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
CAM = dict(width=160, height=120, fx=144.02, fy=144.02, cx=80.27, cy=60.74)


def zhash(z):
    return hashlib.sha256(np.ascontiguousarray(z, np.int32).tobytes()).hexdigest()


def make(name, names, n_poses, stride, seed):
    rng = np.random.default_rng(seed)
    K = len(names)
    gts = np.stack([syn.default_gt_pose(rng, (0.04 * (i - (K - 1) / 2), 0.0, 0.6 + 0.05 * i)) for i in range(K)])

    def rf(tris, cnt, p16, pm, W, H, proj):
        return oracle.render_depth(tris, cnt, p16, pm, None, W, H, proj, np.zeros((H, W), np.int32), None, 1.0)

    sc = syn.make_scene(names, gts, rf, cam=CAM, rng=rng, k=6)
    xyz, _, lab = oracle.depth_to_cloud(sc.depth_raw, stride, sc.cx, sc.cy, sc.fx, sc.fy, sc.depth_factor,
                                        label_mask=sc.mask)
    order = np.argsort(lab, kind="stable")
    oxyz, olab = xyz[order], lab[order]
    ls = np.array([np.searchsorted(olab, L, "left") for L in range(K)], np.int32)
    le = np.array([np.searchsorted(olab, L, "right") for L in range(K)], np.int32)
    poses, pm = [], []
    for k in range(K):
        P = syn.candidate_poses(gts[k][:3, 3], n_poses, rng, include=gts[k], num_viewpoints=20, inplane=4)
        poses.append(init_from_eigen_batch(P))
        pm.append(np.full(len(P), k, np.int32))
    poses = np.concatenate(poses)
    pm = np.concatenate(pm)
    tot = np.bincount(lab, minlength=K).astype(np.float32)[pm]
    src = sc.src_depth_cm
    z = oracle.render_depth(sc.bank.tris, sc.bank.tris_model_count, poses, pm, pm, sc.width, sc.height, sc.proj,
                            src, sc.mask, 1.0)
    rc, oc, df = oracle.evaluate(sc.bank.tris, sc.bank.tris_model_count, poses, pm, pm, sc.width, sc.height,
                                 sc.proj, src, sc.mask, 1.0, stride, sc.cx, sc.cy, sc.fx, sc.fy, 100.0, oxyz, ls, le,
                                 tot, 2, True, 0.01)
    bc, bi = oracle.select(rc, oc, pm, K)
    np.savez_compressed(
        os.path.join(OUT, name), tris=sc.bank.tris, tris_model_count=sc.bank.tris_model_count, poses=poses,
        pose_model=pm, pose_obs_total=tot, proj=sc.proj,
        cam=np.array([sc.width, sc.height, sc.fx, sc.fy, sc.cx, sc.cy], np.float64), stride=np.int32(stride),
        depth_raw=sc.depth_raw, mask=sc.mask, src_depth_cm=src, depth_factor=np.float32(sc.depth_factor),
        obs_xyz=xyz, obs_label=lab, z_hash=np.array([zhash(zi) for zi in z]), z_sum=z.reshape(len(z), -1).sum(1),
        z_first=z[:4], rc=rc, oc=oc, diff=df, best_cost=bc, best_index=bi)
    print(name, len(poses), "poses,", len(xyz), "observed points, best", bc, bi)


if __name__ == "__main__":
    make("oracle_scene_1obj.npz", ["003_cracker_box"], 48, 4, 11)
    make("oracle_scene_3obj.npz", ["003_cracker_box", "005_tomato_soup_can", "061_foam_brick"], 24, 4, 12)
