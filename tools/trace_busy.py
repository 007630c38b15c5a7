#!/usr/bin/env python
"""GPU time per launch of a kernel from a rocprofv3 kernel trace (run_kernel_trace.csv): the union of its
dispatch intervals divided by the dispatches, beside the mean dispatch span (what --stats averages).  With two
batches in flight (bench.py, core.PoseLanes) consecutive dispatches overlap and the two differ.
    python tools/trace_busy.py gpurun_out/prof_r02/run_kernel_trace.csv [kernel-substring] [out.json]"""
import csv
import json
import sys


def main():
    path = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "fused_cost_kernel<8"
    iv = []
    for r in csv.DictReader(open(path)):
        if key in r["Kernel_Name"]:
            iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    iv.sort()
    busy, lo, hi = 0, iv[0][0], iv[0][1]
    for a, b in iv[1:]:
        if a > hi:
            busy += hi - lo
            lo, hi = a, b
        else:
            hi = max(hi, b)
    busy += hi - lo
    res = {"kernel": key, "dispatches": len(iv), "mean_span_ms": sum(b - a for a, b in iv) / len(iv) / 1e6,
           "gpu_ms_per_dispatch": busy / len(iv) / 1e6, "source": path}
    print(json.dumps(res))
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
