#!/usr/bin/env python
"""Small-triangle flush statistics of the fused kernel (C2 workload) from a -DPCORE_FLUSH_STATS build
(PCORE_LIB=build_ab/fst.so), one launch, per pose: flush batches (64 lanes), queued records, fragment tests,
partial flushes forced by the vertex ring or a stream switch, big (cooperative) triangles, triangles touching
a sample, triangle lanes, triangle batches (steps) and vertex passes."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from perception_amd import _native, workloads  # noqa: E402

w = workloads.build(poses_per_model=10000)
w.core.evaluate(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=w.stride)
torch.cuda.synchronize()
L = _native.load()
L.pcore_debug_flush_stats.argtypes = [ctypes.c_void_p]
base = np.zeros(9, dtype=np.uint64)
assert L.pcore_debug_flush_stats(base.ctypes.data) == 0
w.core.evaluate(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=w.stride)
torch.cuda.synchronize()
after = np.zeros(9, dtype=np.uint64)
assert L.pcore_debug_flush_stats(after.ctypes.data) == 0
d = (after - base).astype(np.int64) / 10000.0
names = ["batches", "records", "frag_tests", "forced_flushes", "big_tris", "tris_touching", "tri_lanes", "tri_steps",
         "vertex_passes"]
res = {k: float(v) for k, v in zip(names, d)}
res["lane_util_flush"] = res["records"] / max(res["batches"] * 64, 1)
print(json.dumps({"per_pose": res}))
