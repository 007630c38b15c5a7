#!/usr/bin/env python
"""A larger random-pose parity sweep than the GPU test suite runs (tests/test_gpu_fullsize.py,
test_random_pose_sweep_bit_exact_vs_oracle): --batches batches of --poses random poses each (uniform random rotations;
translations behind, across and near the camera plane, off screen and far, a quarter close to the camera), three
models, scored on the GPU and by the oracle; every pose's rc / oc / diff compared bit for bit.  Optionally the same for
GICP on C3-style candidates (--icp N: N candidates around the five C3 objects, refined poses, iteration counts and costs).
    python tools/parity_sweep.py [--batches 10] [--poses 20000] [--icp 5000] [--out FILE.json]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from perception_amd import synthetic as syn  # noqa: E402
from perception_amd import workloads  # noqa: E402
from perception_amd.model import init_from_eigen_batch  # noqa: E402
from tests.test_gpu_fullsize import _bits, _oracle_poses, _random_poses  # noqa: E402


def sweep_costs(batches, n, cam):
    w = workloads.build(names=["003_cracker_box", "005_tomato_soup_can", "024_bowl"], poses_per_model=10,
                        cam=syn.CAM_640 if cam == "640" else syn.CAM_1280)
    dev = w.poses.device
    totals = {"poses": 0, "mismatching_poses": 0, "visible": 0, "empty": 0}
    for b in range(batches):
        rng = np.random.default_rng(1000 + b)
        p16 = init_from_eigen_batch(_random_poses(rng, n))
        pm = rng.integers(0, w.num_models, n).astype(np.int32)
        tot = np.bincount(w.obs_label.cpu().numpy(), minlength=w.num_models).astype(np.float32)[pm]
        poses, pmt, tott = (torch.from_numpy(p16).to(dev), torch.from_numpy(pm).to(dev),
                            torch.from_numpy(tot).to(dev))
        for _ in range(2):  # the second call runs with the tier the first call's histogram picks
            rc, oc, df = w.core.evaluate(poses, pmt, pmt, tott, stride=w.stride)
        orc, ooc, odf = _oracle_poses(w, p16, pm, tot)
        rc, oc, df = rc.cpu().numpy(), oc.cpu().numpy(), df.cpu().numpy()
        bad = (_bits(rc) != _bits(orc)) | (_bits(oc) != _bits(ooc)) | (_bits(df) != _bits(odf))
        totals["poses"] += n
        totals["mismatching_poses"] += int(bad.sum())
        totals["visible"] += int((rc >= 0).sum())
        totals["empty"] += int((rc < 0).sum())
        print(f"cam {cam} batch {b}: {int(bad.sum())} of {n} differ", file=sys.stderr, flush=True)
    return totals


def sweep_icp(n, windows=(8, 0)):
    """GPU vs oracle for each cycle-exit window (bit for bit), then the exit against running every iteration out
    (DESIGN.md section 5): refined float poses bit-identical or within 1e-6, iteration counts, post-ICP costs and the
    per-model argmin (oracle.select) identical."""
    names = ["003_cracker_box", "005_tomato_soup_can", "006_mustard_bottle", "010_potted_meat_can", "024_bowl"]
    w = workloads.build(names=names, poses_per_model=max(1, n // len(names)), seed=syn.SEED + 17)
    sc = w.scene
    p16 = w.poses.cpu().numpy()
    pm = w.pose_model.cpu().numpy()
    pl = w.pose_label.cpu().numpy()
    tot = w.pose_obs_total.cpu().numpy()
    xyz, lab = w.obs_xyz.cpu().numpy(), w.obs_label.cpu().numpy()
    order = np.argsort(lab, kind="stable")
    oxyz, olab = xyz[order], lab[order]
    nl = int(olab.max()) + 1
    ls = np.array([np.searchsorted(olab, L, "left") for L in range(nl)], np.int32)
    le = np.array([np.searchsorted(olab, L, "right") for L in range(nl)], np.int32)
    cov = np.zeros((len(oxyz), 6))
    for L in range(nl):
        if le[L] > ls[L]:
            cov[ls[L]:le[L]] = oracle.covariances(oxyz[ls[L]:le[L]])
    res = {}
    outs = {}
    for win in windows:
        adj, it, rc, oc, df = w.core.evaluate_icp(w.poses, w.pose_model, w.pose_label, w.pose_obs_total,
                                                  stride=w.stride, cycle_exit_window=win)
        st = w.core.stats()
        print(f"icp window {win}: GPU done, oracle on {len(p16)} candidates", file=sys.stderr, flush=True)
        oadj, oit, orc, ooc, odf = oracle.evaluate_icp(sc.bank.tris, sc.bank.tris_model_count, p16, pm, pl, sc.width,
                                                       sc.height, sc.proj, sc.src_depth_cm, sc.mask, 1.0, w.stride,
                                                       sc.cx, sc.cy, sc.fx, sc.fy, 100.0, oxyz, cov, ls, le, tot, 2,
                                                       True, 0.01, cycle_window=win)
        adj, it = adj.cpu().numpy(), it.cpu().numpy()
        rc, oc, df = rc.cpu().numpy(), oc.cpu().numpy(), df.cpu().numpy()
        bad = ((_bits(adj) != _bits(oadj)).any(1) | (it != oit) | (_bits(rc) != _bits(orc))
               | (_bits(oc) != _bits(ooc)) | (_bits(df) != _bits(odf)))
        res[f"window_{win}"] = {"candidates": int(len(p16)), "mismatching_gpu_vs_oracle": int(bad.sum()),
                                "at_150": int((oit >= 150).sum()), "iterations_mean": float(oit.mean()),
                                "gicp_iterations": int(st["gicp_iterations"]),
                                "gicp_iterations_run": int(st["gicp_iterations_run"]),
                                "gicp_cycle_exits": int(st["gicp_cycle_exits"]), "gicp_ms": float(st["gicp_ms"])}
        outs[win] = (adj, it, rc, oc, df)
    if len(windows) == 2:
        (a1, i1, r1, o1, d1), (a0, i0, r0, o0, d0) = outs[windows[0]], outs[windows[1]]
        ident = ~(_bits(a1) != _bits(a0)).any(1)
        diff = np.abs(a1.astype(np.float64) - a0.astype(np.float64)).max(1)
        scale = np.abs(a0.astype(np.float64)).max(1)
        k1 = oracle.select(r1, o1, pm, len(names))
        k0 = oracle.select(r0, o0, pm, len(names))
        res["exit_vs_full"] = {
            "poses_bit_identical": int(ident.sum()), "poses_bit_identical_frac": float(ident.mean()),
            "max_rel_diff_others": float((diff / np.maximum(scale, 1e-30))[~ident].max()) if (~ident).any() else 0.0,
            "max_abs_diff_others_cm_scaled": float(diff[~ident].max()) if (~ident).any() else 0.0,
            "iterations_equal": bool(np.array_equal(i1, i0)),
            "costs_identical": int(((_bits(r1) == _bits(r0)) & (_bits(o1) == _bits(o0))
                                    & (_bits(d1) == _bits(d0))).sum()),
            "argmin_identical": bool(np.array_equal(k1[0], k0[0]) and np.array_equal(k1[1], k0[1])),
            "argmin": [[int(c), int(i)] for c, i in zip(*k1)]}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=10)
    ap.add_argument("--poses", type=int, default=20000)
    ap.add_argument("--icp", type=int, default=0)
    ap.add_argument("--out")
    a = ap.parse_args()
    t0 = time.time()
    res = {}
    if a.batches > 0:
        res["costs_640"] = sweep_costs(a.batches, a.poses, "640")
        res["costs_1280"] = sweep_costs(max(1, a.batches // 5), a.poses, "1280")
    if a.icp:
        res["icp_c3"] = sweep_icp(a.icp)
    res["seconds"] = time.time() - t0
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
