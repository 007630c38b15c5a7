"""On-disk formats around the hot path.

- PLY meshes (ascii / binary little- and big-endian; vertex x y z [+ red green blue [alpha]]; faces as
  vertex_indices lists, polygons fan-triangulated).  Replaces assimp in Model::LoadModel
  (cuda_renderer/src/model.cpp:16-135): triangle soup in file order, colour of vertex 0 per triangle
  (round(c*255), default 128), node transforms = identity (PLY has no scene graph).
- poses.txt written by the Python harness (fat_pose_image.py:774-775) and read by
  GenerateSuccessorStates (search_env.cpp:7098-7203): one pose per line "x y z qx qy qz qw", metres.
- output_poses.txt / output_stats.txt written by perch_fat (perch_fat.cpp:302-323) and parsed by
  FATPerch.run_perch_node (perch.py:195-230): 13 lines per object.
- 16-bit depth / 8-bit mask PNGs (SetInput, search_env.cpp:5886-5915) via Pillow.
"""
from __future__ import annotations

import hashlib
import os
import time
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from .model import Model

_PLY_TYPES = {
    "char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2", "ushort": "u2",
    "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4", "float": "f4", "float32": "f4",
    "double": "f8", "float64": "f8",
}


@dataclass
class _Element:
    name: str
    count: int
    props: list  # (name, dtype) or (name, ("list", count_dtype, item_dtype))


def _parse_header(f):
    if f.readline().strip() != b"ply":
        raise ValueError("not a PLY file")
    fmt = None
    elements: List[_Element] = []
    while True:
        line = f.readline()
        if not line:
            raise ValueError("truncated PLY header")
        tok = line.strip().split()
        if not tok or tok[0] in (b"comment", b"obj_info"):
            continue
        if tok[0] == b"format":
            fmt = tok[1].decode()
        elif tok[0] == b"element":
            elements.append(_Element(tok[1].decode(), int(tok[2]), []))
        elif tok[0] == b"property":
            if tok[1] == b"list":
                elements[-1].props.append((tok[4].decode(), ("list", _PLY_TYPES[tok[2].decode()],
                                                             _PLY_TYPES[tok[3].decode()])))
            else:
                elements[-1].props.append((tok[2].decode(), _PLY_TYPES[tok[1].decode()]))
        elif tok[0] == b"end_header":
            break
    if fmt not in ("ascii", "binary_little_endian", "binary_big_endian"):
        raise ValueError(f"unsupported PLY format {fmt}")
    return fmt, elements


def _read_binary(f, el: _Element, endian: str):
    if all(not isinstance(t, tuple) for _, t in el.props):
        dt = np.dtype([(n, endian + t) for n, t in el.props])
        return {"__array__": np.frombuffer(f.read(dt.itemsize * el.count), dtype=dt, count=el.count)}
    rows = []
    for _ in range(el.count):
        row = {}
        for n, t in el.props:
            if isinstance(t, tuple):
                cdt = np.dtype(endian + t[1])
                cnt = int(np.frombuffer(f.read(cdt.itemsize), cdt)[0])
                idt = np.dtype(endian + t[2])
                row[n] = np.frombuffer(f.read(idt.itemsize * cnt), idt, count=cnt)
            else:
                d = np.dtype(endian + t)
                row[n] = np.frombuffer(f.read(d.itemsize), d)[0]
        rows.append(row)
    return {"__rows__": rows}


def _read_ascii(f, el: _Element):
    rows = []
    for _ in range(el.count):
        vals = f.readline().split()
        row, k = {}, 0
        for n, t in el.props:
            if isinstance(t, tuple):
                cnt = int(vals[k]); k += 1
                row[n] = np.array([float(v) for v in vals[k:k + cnt]]).astype(t[2]); k += cnt
            else:
                row[n] = np.array(float(vals[k])).astype(t)[()]; k += 1
        rows.append(row)
    return {"__rows__": rows}


def load_ply(path: str, name: Optional[str] = None) -> Model:
    """PLY -> Model with the triangle soup and per-triangle vertex-0 colour (model.cpp:60-99)."""
    with open(path, "rb") as f:
        fmt, elements = _parse_header(f)
        data = {}
        for el in elements:
            if fmt == "ascii":
                data[el.name] = _read_ascii(f, el)
            else:
                data[el.name] = _read_binary(f, el, "<" if fmt == "binary_little_endian" else ">")
    v = data["vertex"]
    if "__array__" in v:
        arr = v["__array__"]
        xyz = np.stack([arr["x"], arr["y"], arr["z"]], 1).astype(np.float32)
        names = arr.dtype.names
        col = None
        if all(c in names for c in ("red", "green", "blue")):
            col = np.stack([arr["red"], arr["green"], arr["blue"]], 1)
    else:
        rows = v["__rows__"]
        xyz = np.array([[r["x"], r["y"], r["z"]] for r in rows], np.float32)
        col = None
        if rows and all(c in rows[0] for c in ("red", "green", "blue")):
            col = np.array([[r["red"], r["green"], r["blue"]] for r in rows])
    faces = data.get("face")
    polys = []
    if faces is not None:
        if "__array__" in faces:
            raise ValueError("face element without a list property")
        key = "vertex_indices" if faces["__rows__"] and "vertex_indices" in faces["__rows__"][0] else "vertex_index"
        polys = [np.asarray(r[key], np.int64) for r in faces["__rows__"]]
    tris, tcol = [], []
    for p in polys:
        if len(p) < 3:
            continue  # model.cpp:76 skips faces with fewer than 3 indices
        for k in range(1, len(p) - 1):  # fan triangulation (assimp Triangulate)
            idx = (p[0], p[k], p[k + 1])
            tris.append(np.concatenate([xyz[i] for i in idx]))
            if col is not None:
                c = col[idx[0]].astype(np.float64)
                if col.dtype.kind == "f":
                    c = np.round(c * 255.0)
                tcol.append(np.clip(c, 0, 255))
    tris = np.asarray(tris, np.float32).reshape(-1, 9)
    colors = np.asarray(tcol, np.uint8).reshape(-1, 3) if col is not None else None
    return Model(name=name or path.rsplit("/", 1)[-1].rsplit(".", 1)[0], tris=tris, colors=colors)


def save_ply(path: str, model: Model, binary: bool = True):
    """Write a Model as an indexed PLY (exact-bit vertex dedupe, per-vertex colour of the first use)."""
    v = model.tris.reshape(-1, 3)
    uniq, inv = np.unique(v.view(np.uint32).reshape(-1, 3), axis=0, return_inverse=True)
    uniq = uniq.view(np.float32).reshape(-1, 3)
    faces = inv.reshape(-1, 3)
    vcol = np.full((len(uniq), 3), 128, np.uint8)
    vcol[faces[:, 0]] = model.colors
    head = ["ply", f"format {'binary_little_endian' if binary else 'ascii'} 1.0", f"element vertex {len(uniq)}",
            "property float x", "property float y", "property float z", "property uchar red",
            "property uchar green", "property uchar blue", f"element face {len(faces)}",
            "property list uchar int vertex_indices", "end_header"]
    with open(path, "wb") as f:
        f.write(("\n".join(head) + "\n").encode())
        if binary:
            vd = np.zeros(len(uniq), dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("r", "u1"), ("g", "u1"),
                                            ("b", "u1")])
            vd["x"], vd["y"], vd["z"] = uniq[:, 0], uniq[:, 1], uniq[:, 2]
            vd["r"], vd["g"], vd["b"] = vcol[:, 0], vcol[:, 1], vcol[:, 2]
            f.write(vd.tobytes())
            fd = np.zeros(len(faces), dtype=[("n", "u1"), ("i", "<i4", 3)])
            fd["n"] = 3
            fd["i"] = faces
            f.write(fd.tobytes())
        else:
            for p, c in zip(uniq, vcol):
                f.write(f"{float(p[0])!r} {float(p[1])!r} {float(p[2])!r} {c[0]} {c[1]} {c[2]}\n".encode())
            for t in faces:
                f.write(f"3 {t[0]} {t[1]} {t[2]}\n".encode())


# ------------------------------------------------------------------------------------------------
# pose lists
# ------------------------------------------------------------------------------------------------

def write_poses_txt(path: str, poses_xyz_qxyzw: np.ndarray, decimals: int = 4):
    """fat_pose_image.py:760-775: np.savetxt(path, np.around(poses, 4)) of rows 'x y z qx qy qz qw'
    (metres), i.e. '%.18e' fields separated by one space."""
    rows = np.asarray(poses_xyz_qxyzw, np.float64).reshape(-1, 7)
    np.savetxt(path, np.around(rows, decimals))


def read_poses_txt(path: str) -> np.ndarray:
    """GenerateSuccessorStates (search_env.cpp:7098-7130): split on ' ', std::stod each field; the first 7
    fields of each line, up to the first empty line.  Files of exactly 7 single-space-separated fields per
    line (what write_poses_txt and the reference's scripts produce) are parsed in one pass; anything else
    line by line."""
    with open(path) as f:
        return _parse_poses_text(f.read())


def _parse_poses_text(text: str) -> np.ndarray:
    lines = text.split("\n")
    end = next((i for i, ln in enumerate(lines) if not ln), len(lines))
    lines = lines[:end]
    fields = " ".join(lines).split(" ")
    if lines and len(fields) == 7 * len(lines) and all(ln.count(" ") == 6 for ln in lines):
        return np.array(fields, dtype=np.float64).reshape(-1, 7)
    rows = [[float(v) for v in ln.split(" ")[:7]] for ln in lines]
    return np.asarray(rows, np.float64).reshape(-1, 7)


try:
    import xxhash as _xxhash

    def _content_digest(data: bytes) -> bytes:
        return _xxhash.xxh3_128_digest(data)
except ImportError:  # pragma: no cover - xxhash ships with the image
    def _content_digest(data: bytes) -> bytes:
        return hashlib.blake2b(data, digest_size=16).digest()


_POSES_CACHE: "OrderedDict[tuple, np.ndarray]" = OrderedDict()
_POSES_CACHE_MAX = 64
_POSES_STAT: "OrderedDict[str, tuple]" = OrderedDict()  # abspath -> (stat signature, content digest)
_SETTLED_NS = 2_000_000_000
# where the file system's clock cannot be measured (no temporary file can be created: a read-only data set), "settled"
# is judged on this host's clock with a wider margin instead
_SETTLED_LOCAL_NS = 60_000_000_000
_FS_CLOCK: dict = {}  # st_dev -> (offset of the file system's clock from time.time_ns or None, time_ns, monotonic_ns)
_FS_CLOCK_TTL_NS = 600_000_000_000


def _fs_clock_offset(directory: str):
    """The file system's clock minus this host's (ns): the ctime of a temporary file created in `directory` against
    time.time_ns() around its creation; None when no file can be created there."""
    import tempfile

    t0 = time.time_ns()
    try:
        fd, tmp = tempfile.mkstemp(prefix=".pcore_clock_", dir=directory)
    except OSError:
        return None
    try:
        ctime = os.fstat(fd).st_ctime_ns
    finally:
        os.close(fd)
        try:
            os.unlink(tmp)
        except OSError:
            pass
    return ctime - (t0 + time.time_ns()) // 2


def _fs_now_ns(directory: str, dev=None):
    """The current time on the clock of the file system holding `directory` (None when it cannot be measured).  The
    clock's offset from this host's is measured once per device (one temporary file, not one per read: ADVICE r05) and
    measured again after 10 minutes, or at once when this host's wall clock stepped (its advance since the measurement
    differs from the monotonic clock's by more than 1 s)."""
    if dev is None:
        dev = os.stat(directory).st_dev
    now, mono = time.time_ns(), time.monotonic_ns()
    ent = _FS_CLOCK.get(dev)
    if ent is None or now - ent[1] > _FS_CLOCK_TTL_NS or abs((now - ent[1]) - (mono - ent[2])) > 1_000_000_000:
        ent = (_fs_clock_offset(directory), now, mono)
        _FS_CLOCK[dev] = ent
    return None if ent[0] is None else now + ent[0]


def _stat_signature(st: os.stat_result) -> tuple:
    return st.st_dev, st.st_ino, st.st_size, st.st_mtime_ns, st.st_ctime_ns


def read_poses_txt_cached(path: str, use_cache: bool = True) -> np.ndarray:
    """read_poses_txt, parsed once per file CONTENT: keyed by (path, 128-bit digest of the bytes), so a poses.txt
    rewritten in place -- whatever its size and timestamps -- is parsed again (the reference re-reads and re-parses it
    every GenerateSuccessorStates; the content, and so the result, is the same).  The digest is XXH3-128 (BLAKE2b
    when xxhash is not importable; BLAKE2b took 1.3-4.7 ms per 10k-pose file).

    A file whose status change time was already 2 s old when it was read is not read again while its (device,
    inode, size, mtime, ctime) stay the same: any write after that read sets ctime to the current time, which no
    utime call can set back, so an unchanged signature means unchanged bytes.  "Now" is the file system's own clock
    (the ctime of a temporary file created beside it), not this host's, so a server clock that lags (NFS) cannot make a
    fresh file look settled.  The file system's clock is this host's plus an offset measured once per
    device (a temporary file per read wrote into the data set); where no temporary file can be created
    (a read-only data set) the host's clock stands in with a 60 s margin.
    A file changed within the last 2 s (the kernel's timestamp clock is coarse) is read and hashed every time.  Least-recently-used eviction past 64
    files.  use_cache=False (or PCORE_POSES_CACHE=0) parses every time.  Returns a read-only array."""
    if not use_cache or os.environ.get("PCORE_POSES_CACHE", "1") == "0":
        return read_poses_txt(path)
    apath = os.path.abspath(path)
    sig = _stat_signature(os.stat(apath))
    known = _POSES_STAT.get(apath)
    if known is not None and known[0] == sig and (apath, known[1]) in _POSES_CACHE:
        key = (apath, known[1])
        _POSES_CACHE.move_to_end(key)
        _POSES_STAT.move_to_end(apath)
        return _POSES_CACHE[key]
    with open(apath, "rb") as f:
        sig_open = _stat_signature(os.fstat(f.fileno()))
        data = f.read()
        sig_read = _stat_signature(os.fstat(f.fileno()))
    key = (apath, _content_digest(data))
    _POSES_STAT.pop(apath, None)
    settled = False
    if sig_open == sig_read:
        fs_now = _fs_now_ns(os.path.dirname(apath), sig_read[0])
        if fs_now is not None:
            settled = fs_now - sig_read[4] > _SETTLED_NS
        else:
            settled = time.time_ns() - sig_read[4] > _SETTLED_LOCAL_NS
    if settled:
        _POSES_STAT[apath] = (sig_read, key[1])
        while len(_POSES_STAT) > _POSES_CACHE_MAX:
            _POSES_STAT.popitem(last=False)
    hit = _POSES_CACHE.get(key)
    if hit is None:
        hit = _parse_poses_text(data.decode())
        hit.setflags(write=False)
        _POSES_CACHE[key] = hit
        while len(_POSES_CACHE) > _POSES_CACHE_MAX:
            _POSES_CACHE.popitem(last=False)
    else:
        _POSES_CACHE.move_to_end(key)
    return hit


# ------------------------------------------------------------------------------------------------
# PERCH outputs
# ------------------------------------------------------------------------------------------------

@dataclass
class DetectedObject:
    name: str
    translation: np.ndarray       # (3,)
    quaternion_xyzw: np.ndarray   # (4,)
    transform: np.ndarray         # 4x4 incl. preprocessing (GetRawModelToSceneTransform)
    preprocessing: np.ndarray     # 4x4


def _mat_lines(m):
    return [" ".join(f"{v:g}" for v in row) for row in np.asarray(m, np.float64).reshape(4, 4)]


def write_output_poses(path: str, objects: Sequence[DetectedObject]):
    """perch_fat.cpp:302-307: 13 lines per object."""
    with open(path, "w") as f:
        for o in objects:
            f.write(o.name + "\n")
            f.write("translation " + " ".join(f"{v:g}" for v in o.translation) + "\n")
            f.write("quaternion " + " ".join(f"{v:g}" for v in o.quaternion_xyzw) + " \n")
            f.write("matrix(incl preprocessing) \n")
            f.write("\n".join(_mat_lines(o.transform)) + "\n")
            f.write("matrix(preprocessing) \n")
            f.write("\n".join(_mat_lines(o.preprocessing)) + "\n")


def read_output_poses(path: str) -> List[DetectedObject]:
    """perch.py:195-218 parser."""
    with open(path) as f:
        lines = f.readlines()
    out = []
    for i in range(0, len(lines) - 12, 13):
        loc = [float(v) for v in lines[i + 1].split()[1:]]
        quat = [float(v) for v in lines[i + 2].split()[1:]]
        T = np.array([[float(v) for v in lines[i + k].split()] for k in range(4, 8)])
        P = np.array([[float(v) for v in lines[i + k].split()] for k in range(9, 13)])
        out.append(DetectedObject(lines[i].rstrip(), np.array(loc), np.array(quat), T, P))
    return out


def write_output_stats(path: str, scenes_rendered: int, scenes_valid: int, expands: int, time_s: float,
                       cost: float, icp_time: float, peak_gpu_mem: float):
    """perch_fat.cpp:316-323."""
    with open(path, "w") as f:
        f.write("[[[[[[[[  Stats  ]]]]]]]]:\n")
        f.write("#Rendered #Valid Rendered #Expands Time Cost ICP-Time Peak-GPU-Mem\n")
        f.write(f"{scenes_rendered} {scenes_valid} {expands} {time_s} {cost} {icp_time} {peak_gpu_mem}\n")


def write_cost_dump(path: str, poses: List[dict]):
    """<debug_dir>/cost_dump.json (search_env.cpp:2463-2464, 2647-2649): {"poses": [...]} as nlohmann::json prints
    it with std::setw(4) -- keys in sorted order (nlohmann's std::map objects), four-space indent, one array element
    per line, floats (stored as double) in shortest round-trip form, and a trailing newline (std::endl).  Read by
    convert_fat_coco.py:1365-1369."""
    import json

    with open(path, "w") as f:
        f.write(json.dumps({"poses": poses}, indent=4, sort_keys=True))
        f.write("\n")


def read_cost_dump(path: str) -> List[dict]:
    """The "poses" list of a cost_dump.json (as convert_fat_coco.py:1368-1369 loads it)."""
    import json

    with open(path) as f:
        return json.load(f)["poses"]


def read_output_stats(path: str) -> Dict[str, float]:
    """perch.py:220-229."""
    with open(path) as f:
        vals = [float(v) for v in f.readlines()[2].split()]
    return {"rendered": vals[0], "expands": vals[2], "runtime": vals[3], "icp_runtime": vals[5],
            "peak_gpu_mem": vals[6]}


# ------------------------------------------------------------------------------------------------
# images
# ------------------------------------------------------------------------------------------------

def load_depth_png(path: str) -> np.ndarray:
    """16-bit depth PNG (cv::IMREAD_ANYDEPTH) -> (H, W) int32 raw sensor units."""
    from PIL import Image

    with Image.open(path) as im:
        return np.asarray(im, dtype=np.uint16).astype(np.int32) if im.mode in ("I;16", "I;16B", "I;16L") \
            else np.asarray(im).astype(np.int32)


def load_mask_png(path: str) -> np.ndarray:
    from PIL import Image

    with Image.open(path) as im:
        a = np.asarray(im)
    if a.ndim == 3:
        a = a[..., 0]
    return a.astype(np.uint8)


def save_png(path: str, img: np.ndarray):
    from PIL import Image

    img = np.asarray(img)
    if img.dtype == np.uint16 or img.dtype.kind in "iu" and img.max(initial=0) > 255:
        Image.fromarray(img.astype(np.uint16)).save(path)
    else:
        Image.fromarray(img.astype(np.uint8)).save(path)

