#!/usr/bin/env python
"""What a longest-first launch order would save on the fused kernel's drain: list scheduling of the measured
per-pose workgroup durations (tools/wg_timeline.py --dump, a PCORE_WG_TIMING build) onto the measured number of
concurrent slots, in index order (what the dispatcher does) and in descending duration order.
Usage: launch_order_sim.py DUMP.npz"""
import heapq
import sys

import numpy as np


def makespan(d, slots):
    h = [0.0] * slots
    heapq.heapify(h)
    end = 0.0
    for x in d:
        t = heapq.heappop(h) + x
        end = max(end, t)
        heapq.heappush(h, t)
    return end


def main(path):
    z = np.load(path)
    st, en, ok = z["start"], z["end"], z["ok"]
    d = (en - st)[ok]
    # concurrency: the most workgroups alive at once
    ev = np.concatenate([np.stack([st[ok], np.ones(ok.sum())], 1), np.stack([en[ok], -np.ones(ok.sum())], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    slots = int(np.max(np.cumsum(ev[:, 1])))
    span = float(en[ok].max() - st[ok].min())
    idx = makespan(d, slots)
    lpt = makespan(np.sort(d)[::-1], slots)
    print({"poses": int(ok.sum()), "slots": slots, "measured_span_us": round(span, 1),
           "sim_index_order_us": round(idx, 1), "sim_longest_first_us": round(lpt, 1),
           "dur_mean_us": round(float(d.mean()), 2), "dur_p99_us": round(float(np.percentile(d, 99)), 2),
           "dur_max_us": round(float(d.max()), 2)})


if __name__ == "__main__":
    main(sys.argv[1])
