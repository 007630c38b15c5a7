"""CPU tests of the perch_fat process seam (perception_amd/perch_fat.py; perch_fat.cpp:39-330, perch.py:75-233):
the parameter server, the defaults, the model bank rows perch.py writes, and the output files read back by the
restated perch.py reader (tests/perch_reader.py).  The GPU run of the executable is tests/test_gpu_perch_fat.py."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from perception_amd import perch_fat as pf
from perception_amd.recognizer import EnvStats, LocalizationResult
from tests.perch_reader import read_perch_outputs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_param_server_merges_like_rosparam(tmp_path):
    env = tmp_path / "env.yaml"
    env.write_text("perch_params:\n  gpu_stride: 8\n  icp_type: 3\n  sensor_resolution_radius: 0.01\n"
                   "search_resolution_translation: 0.05\n")
    run = tmp_path / "run.json"
    run.write_text(json.dumps({"required_object": ["003_cracker_box"], "perch_params": {"use_color_cost": True},
                               "camera_pose": list(range(16))}))
    ps = pf.ParamServer([str(env), str(run), {"perch_params": {"gpu_stride": 4}}])
    assert ps.get("/perch_params/gpu_stride") == 4  # the later source wins, siblings kept
    assert ps.get("/perch_params/icp_type") == 3 and ps.get("/perch_params/use_color_cost") is True
    assert ps.get("/search_resolution_translation") == 0.05 and not ps.has("/perch_params/missing")
    assert ps.get("/nope/deeper", 7) == 7
    p = pf.perch_params(ps)
    assert (p.gpu_stride, p.icp_type, p.sensor_resolution, p.search_resolution) == (4, 3, 0.01, 0.05)
    assert np.array_equal(pf._camera_pose(ps), np.arange(16.0).reshape(4, 4))  # (i, j) = list[j + 4 i]
    assert pf._model_names(ps) == ["003_cracker_box"]
    assert pf._model_names(pf.ParamServer([{"required_object": "024_bowl"}])) == ["024_bowl"]


def test_perch_params_defaults_are_search_env_defaults():
    """Absent keys take search_env.cpp:153-188's defaults (not a config file's)."""
    p = pf.perch_params(pf.ParamServer())
    assert (p.sensor_resolution, p.min_neighbor_points_for_valid_pose, p.gpu_batch_size, p.gpu_stride) == \
        (0.003, 50, 1000, 8)
    assert (p.use_color_cost, p.color_distance_threshold, p.use_cylinder_observed, p.icp_type) == \
        (False, 20.0, True, 0)
    assert (p.gpu_occlusion_threshold, p.depth_median_blur, p.search_resolution) == (1.0, 17, 0.04)


def test_model_bank_rows_as_perch_py_writes_them():
    """perch.py:128-137: [name, path, flipped, False, symmetry, 0.06, 1] per object; object_recognizer.cpp:101-125."""
    rows = [["003_cracker_box", "/m/003/textured.ply", False, False, 0, 0.06, 1],
            ["024_bowl", "/m/024/textured.ply", True, False, 2, 0.06, 1]]
    bank = pf.model_bank(pf.ParamServer([{"model_bank": rows, "mesh_in_mm": True, "mesh_scaling_factor": 0.0275}]))
    assert list(bank) == ["003_cracker_box", "024_bowl"]
    b = bank["024_bowl"]
    assert (b.file, b.flipped, b.symmetry_mode, b.search_resolution, b.mesh_in_mm, b.mesh_scaling_factor) == \
        ("/m/024/textured.ply", True, 2, 0.06, True, 0.0275)
    with pytest.raises(ValueError):
        pf.model_bank(pf.ParamServer([{"model_bank": [["x", "y", False]]}]))


def test_outputs_parse_with_the_perch_py_reader(tmp_path):
    """output_poses.txt / output_stats.txt as the recognizer writes them, read back by perch.py's own parsing:
    translation, quaternion, both matrices, and the stats columns (#Rendered, #Expands = scenes rendered,
    Time, ICP-Time = the GICP stage's time, Peak-GPU-Mem; object_recognizer.cpp:312-318)."""
    from perception_amd.recognizer import ObjectRecognizer

    rng = np.random.default_rng(4)
    T = [np.eye(4), np.eye(4)]
    T[0][:3, 3] = [0.1, -0.2, 0.9]
    T[1][:3, :3] = np.array([[0, -1, 0], [1, 0, 0], [0, 0, 1.0]])
    P = [np.eye(4), np.eye(4)]
    P[0][:3, 3] = rng.normal(scale=0.01, size=3)
    poses = [np.array([0.1, -0.2, 0.9, 0.0, 0.0, 0.0, 1.0]), np.array([0.0, 0.1, 0.8, 0.0, 0.0, 0.7071068, 0.7071068])]
    st = EnvStats(scenes_rendered=32004, scenes_valid=0, time=0.0231, icp_time=0.0189, peak_gpu_mem=812.5)
    res = LocalizationResult(T, P, poses, ["003_cracker_box", "024_bowl"], [3, 7], [11, 20005], st)
    out = tmp_path / "dbg" / "scene_0001"
    ObjectRecognizer.write_outputs(None, res, str(out))
    ann, stats = read_perch_outputs(str(tmp_path / "dbg"), "scene_0001", {"003_cracker_box": 1, "024_bowl": 13})
    assert [a["category_id"] for a in ann] == [1, 13]
    assert np.allclose(ann[0]["location"], [10.0, -20.0, 90.0])
    assert np.allclose(ann[1]["quaternion_xyzw"], poses[1][3:], atol=1e-6)
    assert np.allclose(ann[1]["transform_matrix"], T[1]) and np.allclose(ann[0]["preprocessing_transform_matrix"],
                                                                         P[0], atol=1e-5)
    assert stats == {"expands": 32004.0, "rendered": 32004.0, "runtime": 0.0231, "icp_runtime": 0.0189,
                     "peak_gpu_mem": 812.5}


def test_compute_type_outside_the_hot_path_exits_2(tmp_path):
    params = tmp_path / "p.yaml"
    params.write_text(f"compute_type: 0\nperch_debug_dir: {tmp_path}\n")
    r = subprocess.run([sys.executable, "-m", "perception_amd.perch_fat", "scene", "--params", str(params)],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "compute_type 0" in r.stderr
