#!/usr/bin/env python
"""GPU time per launch of the bench's timed C2 launches from a rocprofv3 kernel trace (run_kernel_trace.csv).

A profiled `bench.py` run dispatches `fused_cost_kernel<8, ...>` for more than the timed region: one launch that
measures P_r, the warm-ups (unoverlapped, slower), the 20 timed launches, and then the C3 leg's re-score launches over
50 k poses (a grid 5x larger).  Only the timed launches are the time base of the bench line's roofline, so this keeps
the dispatches whose grid equals the C2 launch's (the most common grid of the kernel, or --grid) and of those the last
--last (the bench's --steps; the timed region is the last C2 work before the C3 leg).  It reports:
  mean_span_ms         the mean dispatch span (what rocprofv3 --stats averages; with two batches in flight consecutive
                       dispatches overlap, so this counts shared time twice)
  gpu_ms_per_dispatch  the union of the selected dispatch intervals / dispatches (bench.py's gpu_ms_per_launch)
and, with --sq profiles/sq_counters.json, the VALU roofline recomputed from these tracked files alone.
    python tools/trace_busy.py TRACE.csv [--kernel fused_cost_kernel<8] [--last 20] [--grid G] [--sq SQ.json]
                               [--poses 10000] [--out OUT.json] [--stats-out STATS.csv]"""
import argparse
import collections
import csv
import json

VALU_PEAK = 1024 * 2.4e9 / 2.0  # wave64 VALU instructions per second (bench.py)


def union_ms(iv):
    iv = sorted(iv)
    busy, lo, hi = 0, iv[0][0], iv[0][1]
    for a, b in iv[1:]:
        if a > hi:
            busy += hi - lo
            lo, hi = a, b
        else:
            hi = max(hi, b)
    return (busy + hi - lo) / 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="fused_cost_kernel<8")
    ap.add_argument("--last", type=int, default=20, help="the bench's timed steps (its --steps)")
    ap.add_argument("--grid", type=int, default=None, help="Grid_Size_X of the C2 launch (default: the most common)")
    ap.add_argument("--sq", default=None, help="profiles/sq_counters.json: recompute achieved / frac")
    ap.add_argument("--poses", type=int, default=10000)
    ap.add_argument("--out", default=None)
    ap.add_argument("--stats-out", default=None, help="write a rocprofv3-style stats row of the selected dispatches")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    grids = collections.Counter(int(r["Grid_Size_X"]) for r in rows)
    grid = a.grid if a.grid is not None else grids.most_common(1)[0][0]
    sel = [r for r in rows if int(r["Grid_Size_X"]) == grid][-a.last:]
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in sel]
    spans = [(b - s) / 1e6 for s, b in iv]
    busy = union_ms(iv) / len(iv)
    res = {"kernel": a.kernel, "grid_size_x": grid, "dispatches_of_kernel": len(rows),
           "grids_seen": {str(k): v for k, v in sorted(grids.items())}, "dispatches": len(sel),
           "dispatch_ids": [int(r["Dispatch_Id"]) for r in sel], "mean_span_ms": sum(spans) / len(spans),
           "min_span_ms": min(spans), "max_span_ms": max(spans), "gpu_ms_per_dispatch": busy,
           "selection": f"dispatches with Grid_Size_X == {grid}, the last {a.last} (the bench's timed region)",
           "source": a.trace}
    if a.sq:
        sq = json.load(open(a.sq))
        ipp = float(sq["fused_cost"]["derived_valu_instr_per_pose"])
        ach = ipp * a.poses / (busy * 1e-3)
        res["roofline_from_tracked_files"] = {
            "valu_instr_per_pose": ipp, "poses_per_launch": a.poses, "achieved_Gwave_instr_per_s": ach / 1e9,
            "peak_Gwave_instr_per_s": VALU_PEAK / 1e9, "frac": ach / VALU_PEAK, "sq_source": a.sq,
            "kernel_source_digest": sq.get("kernel_source_digest")}
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    if a.stats_out:
        with open(a.stats_out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "UnionPerCallNs"])
            w.writerow([sel[0]["Kernel_Name"], len(sel), int(sum(spans) * 1e6), int(sum(spans) / len(spans) * 1e6),
                        int(min(spans) * 1e6), int(max(spans) * 1e6), int(busy * 1e6)])


if __name__ == "__main__":
    main()
