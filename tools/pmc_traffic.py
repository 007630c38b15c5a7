#!/usr/bin/env python
"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) into per-launch HBM bytes of the fused
kernel at the bench batch size (median launch).  gfx950 corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE / WRITE_SIZE
are in KiB; FETCH_SIZE reports half the bytes of wide coalesced reads, so it is doubled (an upper bound
for narrower accesses).  Writes profiles/pmc_traffic.json."""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from perception_amd.build import kernel_source_digest  # noqa: E402


def load(path, counter):
    by_grid = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if "fused_cost_kernel" in row["Kernel_Name"] and row["Counter_Name"] == counter:
                by_grid[int(row["Grid_Size"])].append(float(row["Counter_Value"]))
    return by_grid


def main(fetch_csv, write_csv, out, poses_per_launch=10000, threads=256):
    grid = poses_per_launch * threads
    f = load(fetch_csv, "FETCH_SIZE")[grid]
    w = load(write_csv, "WRITE_SIZE")[grid]
    # median over launches: bench.py's first launch also writes the P_r debug z-samples
    fetch_kib = sorted(f)[len(f) // 2]
    write_kib = sorted(w)[len(w) // 2]
    res = {
        "poses_per_launch": poses_per_launch,
        "fetch_size_kib_raw": fetch_kib,
        "write_size_kib": write_kib,
        "hbm_bytes_per_launch": (2.0 * fetch_kib + write_kib) * 1024.0,
        "launches": [len(f), len(w)],
        "note": "FETCH_SIZE doubled per the gfx950 calibration; WRITE_SIZE as reported",
        "kernel_source_digest": kernel_source_digest(),
    }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:4])
