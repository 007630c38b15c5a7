"""Pose-accuracy metrics of the YCB harness.

- ADD / ADD-S of estimated against ground-truth poses over a model's points: compare_clouds
  (fat_pose_image.py:2020-2139) and pose_error.add / adi (lib/utils/pose_error.py:72-108).  The O(n^2)
  ADD-S minimum runs on the GPU (pcore_pose_distances, pcore_metrics.hip) in f64 -- the reference runs
  sklearn's pairwise_distances_argmin_min on the CPU.
- compute_pose_metrics (fat_pose_image.py:3793-3833): ADD-S AUC up to 10 cm, the share of poses under
  2 cm and the mean error, following YCB_Video_toolbox plot_accuracy_keyframe.m.
- match_detections: the per-detection ground-truth choice of compare_clouds (2026-2048): same category,
  nearest location.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .core import PoseCore, _ptr, _stream


def rt_to_matrix(R: np.ndarray, t: np.ndarray) -> np.ndarray:
    T = np.eye(4)
    T[:3, :3] = np.asarray(R, np.float64)
    T[:3, 3] = np.asarray(t, np.float64).reshape(3)
    return T


def pose_distances(core: PoseCore, pts, T_gt, T_est, adds: bool = True, stream=None
                   ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """ADD (and ADD-S) for every pair (T_gt[m], T_est[m]) over the model points `pts` (n x 3).

    `pts` float32, `T_gt` / `T_est` (M, 4, 4) float64; numpy arrays are copied to the core's device,
    GPU tensors are used in place.  Returns (add, adds) float64 tensors of length M on the device."""
    dev = torch.device("cuda", core.device)
    P = torch.as_tensor(pts, dtype=torch.float32).reshape(-1, 3).to(dev).contiguous()
    G = torch.as_tensor(T_gt, dtype=torch.float64).reshape(-1, 16).to(dev).contiguous()
    E = torch.as_tensor(T_est, dtype=torch.float64).reshape(-1, 16).to(dev).contiguous()
    if G.shape != E.shape:
        raise ValueError("T_gt and T_est must have the same number of poses")
    M = int(G.shape[0])
    add = torch.empty(M, dtype=torch.float64, device=dev)
    out_s = torch.empty(M, dtype=torch.float64, device=dev) if adds else None
    core._check(core.lib.pcore_pose_distances(
        core._h, _ptr(P, torch.float32, "pts"), int(P.shape[0]), _ptr(G, torch.float64, "T_gt"),
        _ptr(E, torch.float64, "T_est"), M, _ptr(add, torch.float64, "add"),
        _ptr(out_s, torch.float64, "adds") if adds else None, _stream(stream)))
    return add, out_s


def add(core: PoseCore, R_est, t_est, R_gt, t_gt, pts) -> float:
    """pose_error.add (pose_error.py:72-86), on the GPU."""
    a, _ = pose_distances(core, pts, rt_to_matrix(R_gt, t_gt)[None], rt_to_matrix(R_est, t_est)[None], adds=False)
    return float(a[0].item())


def adi(core: PoseCore, R_est, t_est, R_gt, t_gt, pts) -> float:
    """pose_error.adi = ADD-S (pose_error.py:89-108): mean over ground-truth points of the distance to
    the nearest estimated point (exact minimum), on the GPU."""
    _, s = pose_distances(core, pts, rt_to_matrix(R_gt, t_gt)[None], rt_to_matrix(R_est, t_est)[None])
    return float(s[0].item())


def compute_pose_metrics(rec, max_auc_dist: float = 0.1, max_pose_dist: float = 0.02) -> Dict[str, float]:
    """fat_pose_image.py:3793-3833 (plot_accuracy_keyframe.m of YCB_Video_toolbox).

    rec: ADD-S (or ADD) errors in metres, one per pose.  Errors above `max_auc_dist` count as misses.
    The curve's right end stays at 0.1 and the area is scaled by 10, as in the reference, whatever
    `max_auc_dist` is.  Unlike the reference, the caller's array is not modified in place."""
    rec = np.array(rec, dtype=np.float64)
    n = rec.shape[0]
    mean = float(np.mean(rec))
    less_perc = np.where(rec < max_pose_dist)[0].shape[0] / n * 100.0
    rec[rec > max_auc_dist] = np.inf
    rec = np.sort(rec)
    prec = np.arange(0, n, 1) / n
    prec = np.array(prec[1:].tolist() + [1])
    keep = np.isfinite(rec)
    rec = rec[keep]
    prec = prec[keep]
    mrec = np.array([0] + rec.tolist() + [0.1])
    mpre = np.array([0] + prec.tolist() + [prec[-1]])
    i = np.where(mrec[:-1] != mrec[1:])[0]
    ap = np.sum((mrec[i + 1] - mrec[i]) * mpre[i + 1]) * 10
    return {"auc": ap * 100.0, "pose_error_less_perc": less_perc, "mean_pose_error": mean,
            "pose_count": rec.shape[0]}


def match_detections(gt: Sequence[dict], est: Sequence[dict]) -> List[Tuple[int, int]]:
    """compare_clouds' pairing (fat_pose_image.py:2026-2048): for every estimate, the ground-truth
    annotation of the same category_id with the nearest 'location' (first on ties); estimates without a
    same-category ground truth are skipped (false positives).  Returns (gt index, est index) pairs."""
    out = []
    for j, e in enumerate(est):
        best, best_d = None, 10000
        for i, g in enumerate(gt):
            if g["category_id"] != e["category_id"]:
                continue
            d = np.linalg.norm(np.array(g["location"]) - np.array(e["location"]))
            if d < best_d:
                best, best_d = i, d
        if best is not None:
            out.append((best, j))
    return out
