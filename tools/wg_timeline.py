#!/usr/bin/env python
"""Workgroup timeline of fused_cost_kernel (C2 workload) from a -DPCORE_WG_TIMING build
(PCORE_LIB=build_ab/wgt.so): per-pose start / end wall clocks (100 MHz) of the last of a few launches.
Prints the span, the duration distribution, and how the span splits into ramp-up (until every slot has
started once), steady state and the tail after the last workgroup started."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from perception_amd import _native, workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--poses", type=int, default=10000)
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--dump", default="")
    a = ap.parse_args()
    w = workloads.build(poses_per_model=a.poses)
    n = int(w.poses.shape[0])
    for _ in range(a.iters):
        w.core.evaluate(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=w.stride)
        torch.cuda.synchronize()
    L = _native.load()
    buf = np.zeros(2 * n, dtype=np.uint64)
    L.pcore_debug_wg_clock.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert L.pcore_debug_wg_clock(buf.ctypes.data, n) == 0
    st = buf[0::2].astype(np.int64)
    en = buf[1::2].astype(np.int64)
    ok = en > 0  # overflow poses return before the end clock of this kernel
    t0 = st.min()
    st, en = (st - t0) / 100.0, (en - t0) / 100.0  # us
    dur = (en - st)[ok]
    span = en[ok].max()
    order = np.sort(st)
    res = {
        "poses": n, "timed": int(ok.sum()), "span_us": float(span),
        "dur_us": {q: float(np.percentile(dur, p)) for q, p in (("p0", 0), ("p10", 10), ("p50", 50), ("p90", 90),
                                                                   ("p99", 99), ("max", 100))},
        "dur_mean_us": float(dur.mean()),
        "last_start_us": float(order[-1]),
        "tail_after_last_start_us": float(span - order[-1]),
        "start_at_slot_1536_us": float(order[min(1535, n - 1)]),
        "mean_concurrency": float(dur.sum() / span),
        "max_concurrency": int(max(((st <= t) & (en > t)).sum() for t in np.arange(0.0, span, 1.0))),
        "tier_env": os.environ.get("PCORE_FUSED_TIER", ""),
        "first_round_dur_mean_us": float(dur[np.argsort(st[ok])[:1536]].mean()),
        "last_round_dur_mean_us": float(dur[np.argsort(st[ok])[-1536:]].mean()),
    }
    # duration against pose window size proxy: correlation with pose index order
    print(json.dumps(res), flush=True)
    if a.dump:
        np.savez_compressed(a.dump, start=st, end=en, ok=ok)


if __name__ == "__main__":
    main()
