"""The YCB evaluation script's reader of perch_fat's outputs, restated from perch.py:195-233 (FATPerch.run_perch_node
after the subprocess returns) for the tests: 13 lines per object, the stats line split on whitespace.  Test
infrastructure (the reference's Python does not import here: ROS)."""
from __future__ import annotations

import os

import numpy as np


def read_perch_outputs(perch_debug_dir: str, output_dir_name: str, object_names_to_id: dict, distance_scale=100):
    """-> (annotations, stats) exactly as perch.py:195-229 builds them; (None, None) for an empty output_poses.txt."""
    annotations = []
    with open(os.path.join(perch_debug_dir, output_dir_name, "output_poses.txt"), "r") as f:
        lines = f.readlines()
    if len(lines) == 0:
        return None, None
    for i in np.arange(0, len(lines), 13):
        location = list(map(float, lines[i + 1].rstrip().split()[1:]))
        quaternion = list(map(float, lines[i + 2].rstrip().split()[1:]))
        transform_matrix = np.zeros((4, 4))
        preprocessing_transform_matrix = np.zeros((4, 4))
        for l_t in range(4, 8):
            transform_matrix[l_t - 4, :] = list(map(float, lines[i + l_t].rstrip().split()))
        for l_t in range(9, 13):
            preprocessing_transform_matrix[l_t - 9, :] = list(map(float, lines[i + l_t].rstrip().split()))
        annotations.append({
            "location": [location[0] * distance_scale, location[1] * distance_scale, location[2] * distance_scale],
            "quaternion_xyzw": quaternion,
            "category_id": object_names_to_id[lines[i].rstrip()],
            "transform_matrix": transform_matrix,
            "preprocessing_transform_matrix": preprocessing_transform_matrix,
            "id": i % 13,
        })
    with open(os.path.join(perch_debug_dir, output_dir_name, "output_stats.txt"), "r") as f:
        lines = f.readlines()
    stats_from_file = list(map(float, lines[2].rstrip().split()))
    stats = {"expands": stats_from_file[2], "rendered": stats_from_file[0], "runtime": stats_from_file[3],
             "icp_runtime": stats_from_file[5], "peak_gpu_mem": stats_from_file[6]}
    return annotations, stats
