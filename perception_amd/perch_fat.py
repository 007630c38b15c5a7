"""perch_fat's process seam: the executable the YCB / FAT evaluation scripts run (perch.py:177-233).

    python -m perception_amd.perch_fat <output_dir_name> [--params FILE ...]
    python -m torch.distributed.run --nproc-per-node N -m perception_amd.perch_fat <output_dir_name> --params ...

Restates sbpl_perception/experiments/src/perch_fat.cpp:39-330 on this build's ObjectRecognizer:
  - the parameters come from a parameter server.  The reference reads ROS params that perch.py put there with
    `rosparam load <env / planner config>` and `rosparam set / "<dict>"` (perch.py:75-99); here every --params FILE
    (YAML or JSON; also the os.pathsep-separated list in $PERCH_PARAMS) is merged into one dict in order, with the
    same semantics: a file's top-level keys become /key, nested mappings (perch_params) become /perch_params/...;
  - experiment_dir = /perch_debug_dir + "/" + stem(output_dir_name) + "/" is removed and re-created by the master
    (perch_fat.cpp:76-107), every rank waits at a barrier;
  - the RecognitionInput fields of perch_fat.cpp:128-176 (x/y bounds, table_height, use_external_pose_list,
    input_color_image, input_depth_image, predicted_mask_image, depth_factor, use_icp, rendered_root_dir,
    camera_pose as 16 row-major values, required_object = the model names), the model bank of
    object_recognizer.cpp:93-130 (7-field rows: name, file, flipped, symmetric, symmetry_mode, search_resolution,
    num_variants; mesh_in_mm, mesh_scaling_factor), the camera of object_recognizer.cpp:57-77 and perch_params with
    the defaults of search_env.cpp:153-188;
  - compute_type 1 = LocalizeObjectsGreedyRender: 6-DoF (use_external_pose_list 1, poses.txt lists) through
    ObjectRecognizer, 3-DoF (0, the table grid) through TabletopRecognizer.  compute_type 0 / 2 (CPU greedy ICP,
    PERCH 1.0 tree search) are outside this build's hot path and exit with status 2;
  - the master writes output_poses.txt (13 lines per detected object) and output_stats.txt (perch_fat.cpp:302-323),
    with the GICP stage's own time (gpu_stats.icp_runtime, search_env.cpp:1715-1716) in the ICP-Time column.

With torch.distributed initialised from the environment (torchrun), every rank searches its contiguous shard of the
candidate states and only rank 0 writes -- the reference's boost::mpi ranks, as one rank per GPU.
"""
from __future__ import annotations

import argparse
import os
import shutil
import sys
import time
from typing import Any, Dict, Iterable, List, Optional

import numpy as np

# search_env.cpp:153-188: /perch_params/<key> -> (PerchParams field, default)
PERCH_PARAM_DEFAULTS = {
    "sensor_resolution_radius": ("sensor_resolution", 0.003),
    "min_neighbor_points_for_valid_pose": ("min_neighbor_points_for_valid_pose", 50),
    "gpu_batch_size": ("gpu_batch_size", 1000),
    "gpu_stride": ("gpu_stride", 8.0),
    "use_color_cost": ("use_color_cost", False),
    "color_distance_threshold": ("color_distance_threshold", 20.0),
    "use_cylinder_observed": ("use_cylinder_observed", True),
    "gpu_occlusion_threshold": ("gpu_occlusion_threshold", 1.0),
    "depth_median_blur": ("depth_median_blur", 17.0),
    "icp_type": ("icp_type", 0),
    "use_model_specific_search_resolution": ("use_model_specific_search_resolution", False),
}
# object_recognizer.cpp:57-77
CAMERA_DEFAULTS = {"camera_width": 640, "camera_height": 480, "camera_fx": 576.09757860, "camera_fy": 576.09757860,
                   "camera_cx": 321.06398107, "camera_cy": 242.97676897}


class ParamServer:
    """The subset of the ROS parameter server perch_fat reads: one nested dict, filled by merging mappings at the
    root (`rosparam load FILE` / `rosparam set / DICT`), read by '/'-separated names."""

    def __init__(self, sources: Iterable[Any] = ()):
        self.root: Dict[str, Any] = {}
        for src in sources:
            self.merge(src)

    @staticmethod
    def _merge(dst: dict, src: dict):
        for k, v in src.items():
            if isinstance(v, dict) and isinstance(dst.get(k), dict):
                ParamServer._merge(dst[k], v)
            else:
                dst[k] = v

    def merge(self, src):
        """A mapping, or the path of a YAML / JSON file holding one."""
        if isinstance(src, (str, os.PathLike)):
            import yaml

            with open(src) as f:
                src = yaml.safe_load(f) or {}
        if not isinstance(src, dict):
            raise ValueError(f"parameter source is not a mapping: {type(src).__name__}")
        self._merge(self.root, src)

    def has(self, name: str) -> bool:
        return self._lookup(name)[0]

    def get(self, name: str, default=None):
        ok, v = self._lookup(name)
        return v if ok else default

    def _lookup(self, name: str):
        node = self.root
        for part in [p for p in name.split("/") if p]:
            if not isinstance(node, dict) or part not in node:
                return False, None
            node = node[part]
        return True, node


def perch_params(ps: ParamServer):
    from .recognizer import PerchParams

    kw = {}
    for key, (field, default) in PERCH_PARAM_DEFAULTS.items():
        v = ps.get(f"/perch_params/{key}", default)
        like = getattr(PerchParams, field)  # the field's type (the dataclass default)
        kw[field] = bool(v) if isinstance(like, bool) else type(like)(v)
    kw["search_resolution"] = float(ps.get("/search_resolution_translation", 0.04))
    return PerchParams(**kw)


def model_bank(ps: ParamServer):
    """object_recognizer.cpp:93-130 (7-field rows) with mesh_in_mm / mesh_scaling_factor."""
    from .recognizer import ModelMetaData

    rows = ps.get("/model_bank")
    if not isinstance(rows, list):
        raise ValueError("/model_bank must be a list of [name, file, flipped, symmetric, symmetry_mode, "
                         "search_resolution, num_variants] rows")
    mm = bool(ps.get("/mesh_in_mm", False))
    scale = float(ps.get("/mesh_scaling_factor", 1.0))
    bank = {}
    for row in rows:
        if not isinstance(row, (list, tuple)) or len(row) != 7:
            raise ValueError(f"model_bank row needs 7 fields: {row!r}")
        name, path, flipped, symmetric, sym_mode, res, _variants = row
        bank[str(name)] = ModelMetaData(str(name), file=str(path), flipped=bool(flipped), symmetric=bool(symmetric),
                                        symmetry_mode=int(sym_mode), search_resolution=float(res), mesh_in_mm=mm,
                                        mesh_scaling_factor=scale)
    return bank


def _model_names(ps: ParamServer) -> List[str]:
    names = ps.get("/required_object", [])
    return [names] if isinstance(names, str) else [str(n) for n in names]


def _camera_pose(ps: ParamServer) -> np.ndarray:
    v = ps.get("/camera_pose")
    if v is None:
        raise ValueError("/camera_pose (16 values, row-major) is required")
    v = np.asarray(v, np.float64).reshape(-1)
    if v.size != 16:
        raise ValueError("/camera_pose needs 16 values")
    return v.reshape(4, 4)  # camera_pose(i, j) = list[j + 4 i] (perch_fat.cpp:157-162)


def _read_image(path: str) -> np.ndarray:
    from PIL import Image

    with Image.open(path) as im:
        if im.mode in ("I;16", "I;16B", "I;16L"):
            return np.asarray(im, dtype=np.uint16).astype(np.int32)
        return np.asarray(im)


def run(output_dir_name: str, ps: ParamServer, device: Optional[int] = None) -> int:
    import torch

    from . import distributed as pdist
    from . import io as pio
    from .recognizer import CameraIntrinsics, ObjectRecognizer, RecognitionInput

    pdist.init_from_env()
    world = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
    rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
    master = rank == 0
    compute_type = int(ps.get("/compute_type", 1))
    if compute_type != 1:
        if master:
            print(f"perch_fat: compute_type {compute_type} (0 = greedy CPU ICP, 2 = PERCH 1.0 tree search) is not "
                  f"part of this build; only 1 (LocalizeObjectsGreedyRender) is", file=sys.stderr)
        return 2
    debug_dir = str(ps.get("/perch_debug_dir", os.path.join(os.getcwd(), "visualization")))
    stem = os.path.splitext(os.path.basename(os.path.normpath(output_dir_name)))[0]
    experiment_dir = os.path.join(debug_dir, stem)
    if master:
        if os.path.isdir(experiment_dir):
            shutil.rmtree(experiment_dir)
        os.makedirs(experiment_dir, exist_ok=True)
    if world > 1:
        torch.distributed.barrier()

    if device is None:
        device = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(device)
    cam = CameraIntrinsics(int(ps.get("/camera_width", CAMERA_DEFAULTS["camera_width"])),
                           int(ps.get("/camera_height", CAMERA_DEFAULTS["camera_height"])),
                           float(ps.get("/camera_fx", CAMERA_DEFAULTS["camera_fx"])),
                           float(ps.get("/camera_fy", CAMERA_DEFAULTS["camera_fy"])),
                           float(ps.get("/camera_cx", CAMERA_DEFAULTS["camera_cx"])),
                           float(ps.get("/camera_cy", CAMERA_DEFAULTS["camera_cy"])))
    params = perch_params(ps)
    bank = model_bank(ps)
    names = _model_names(ps)
    missing = [n for n in names if n not in bank]
    if missing:
        raise ValueError(f"required_object not in model_bank: {missing}")
    camera_pose = _camera_pose(ps)
    depth_factor = float(ps.get("/depth_factor", 10000.0))
    use_external_pose_list = int(ps.get("/use_external_pose_list", 0))
    t0 = time.perf_counter()
    if use_external_pose_list == 1:  # 6-DoF: 16-bit depth, label mask, poses.txt lists
        rec = ObjectRecognizer(bank, cam, params, device)
        rec.debug_dir = experiment_dir  # SetDebugDir (perch_fat.cpp:116): cost_dump.json goes there
        inp = RecognitionInput(names, str(ps.get("/input_depth_image")), str(ps.get("/predicted_mask_image")),
                               depth_factor=depth_factor, camera_pose=camera_pose,
                               rendered_root_dir=ps.get("/rendered_root_dir"),
                               use_external_pose_list=1, use_icp=int(ps.get("/use_icp", 1)))
        result = rec.localize_objects_greedy_render(inp)
    else:  # 3-DoF table-top grid: 8-bit (medianBlur) or 16-bit depth, BGR colour as cv::imread delivers it
        from .tabletop import TableParams, TabletopRecognizer

        table = TableParams(float(ps.get("/x_min", 0.0)), float(ps.get("/x_max", 0.0)), float(ps.get("/y_min", 0.0)),
                            float(ps.get("/y_max", 0.0)), float(ps.get("/table_height", 0.0)),
                            res=float(ps.get("/search_resolution_translation", 0.04)),
                            theta_res=float(ps.get("/search_resolution_yaw", 0.3926991)))
        rec = TabletopRecognizer(bank, cam, table, params, device)
        rec.debug_dir = experiment_dir
        depth = _read_image(str(ps.get("/input_depth_image")))
        rgb = None
        colour = ps.get("/input_color_image")
        if params.use_color_cost and colour:
            img = _read_image(str(colour))
            rgb = np.ascontiguousarray(img[..., :3][..., ::-1]) if img.ndim == 3 else None
        res = rec.localize(names, depth, camera_pose, depth_factor, rgb)
        result = rec.localization_result(res)
    elapsed = time.perf_counter() - t0
    if world > 1:
        torch.distributed.barrier()
    if master:
        rec.write_outputs(result, experiment_dir)
        for name, T in zip(result.model_names, result.object_transforms):
            print(f"Pose for Object: {name}\n{np.array2string(np.asarray(T), precision=6)}\n", flush=True)
        print(f"perch_fat: {len(result.model_names)} objects, {result.stats.scenes_rendered} scenes rendered, "
              f"{elapsed:.3f} s -> {experiment_dir}", flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="perch_fat", description=__doc__.split("\n\n")[0])
    ap.add_argument("output_dir_name")
    ap.add_argument("--params", action="append", default=[],
                    help="YAML / JSON parameter file merged at the root, in order (rosparam load / set /)")
    ap.add_argument("--device", type=int, default=None)
    args = ap.parse_args(argv)
    sources = [p for p in os.environ.get("PERCH_PARAMS", "").split(os.pathsep) if p] + args.params
    return run(args.output_dir_name, ParamServer(sources), args.device)


if __name__ == "__main__":
    sys.exit(main())
