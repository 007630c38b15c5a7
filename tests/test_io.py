"""File formats around the hot path (f2): PLY meshes, poses.txt, output_poses.txt / output_stats.txt,
16-bit depth PNGs (the reference's own demo_depth.png, copied as a data fixture)."""
import os

import numpy as np

import oracle
from perception_amd import io, synthetic as syn
from perception_amd.model import Model

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _per_vertex_colored(model):
    v = model.tris.reshape(-1, 3)
    key = (np.abs(v * 1000).astype(np.int64) % 256)
    model.colors = key.reshape(-1, 3, 3)[:, 0, :].astype(np.uint8)
    return model


def test_ply_roundtrip_binary_and_ascii(tmp_path):
    m = _per_vertex_colored(syn.ycb_proxy("005_tomato_soup_can"))
    for binary in (True, False):
        p = str(tmp_path / f"m{int(binary)}.ply")
        io.save_ply(p, m, binary=binary)
        m2 = io.load_ply(p)
        assert np.array_equal(m2.tris, m.tris)
        assert np.array_equal(m2.colors, m.colors)


def test_ply_polygons_are_fan_triangulated_and_float_colors_rounded(tmp_path):
    p = str(tmp_path / "quad.ply")
    with open(p, "w") as f:
        f.write("ply\nformat ascii 1.0\ncomment test\nelement vertex 4\nproperty float x\nproperty float y\n"
                "property float z\nproperty float red\nproperty float green\nproperty float blue\n"
                "element face 2\nproperty list uchar int vertex_indices\nend_header\n"
                "0 0 0 1 0.5 0\n1 0 0 0 0 0\n1 1 0 0 0 0\n0 1 0 0 0 0\n4 0 1 2 3\n2 0 1\n")
    m = io.load_ply(p)
    assert m.tris.shape == (2, 9)  # quad -> 2 triangles, 2-index face skipped (model.cpp:76)
    assert np.array_equal(m.tris[1], np.array([0, 0, 0, 1, 1, 0, 0, 1, 0], np.float32))
    assert list(m.colors[0]) == [255, 128, 0]


def test_default_color_is_128(tmp_path):
    p = str(tmp_path / "t.ply")
    with open(p, "w") as f:
        f.write("ply\nformat ascii 1.0\nelement vertex 3\nproperty float x\nproperty float y\nproperty float z\n"
                "element face 1\nproperty list uchar int vertex_indices\nend_header\n0 0 0\n1 0 0\n0 1 0\n3 0 1 2\n")
    m = io.load_ply(p)
    assert (m.colors == 128).all()


def test_poses_txt_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    P = np.concatenate([rng.uniform(-1, 1, (50, 3)), rng.normal(size=(50, 4))], 1)
    p = str(tmp_path / "poses.txt")
    io.write_poses_txt(p, P)
    Q = io.read_poses_txt(p)
    assert Q.shape == (50, 7)
    assert np.allclose(Q, P, atol=5e-5)


def test_output_poses_and_stats_roundtrip(tmp_path):
    objs = []
    for i, name in enumerate(["003_cracker_box", "005_tomato_soup_can"]):
        T = np.eye(4)
        T[:3, 3] = (0.1 * i, -0.2, 0.8)
        P = np.eye(4)
        P[:3, 3] = (0, 0, -0.01 * i)
        objs.append(io.DetectedObject(name, T[:3, 3], np.array([0, 0, 0.3, 0.95]), T, P))
    p = str(tmp_path / "output_poses.txt")
    io.write_output_poses(p, objs)
    with open(p) as f:
        assert len(f.readlines()) == 26
    back = io.read_output_poses(p)
    assert [o.name for o in back] == ["003_cracker_box", "005_tomato_soup_can"]
    for a, b in zip(objs, back):
        assert np.allclose(a.transform, b.transform) and np.allclose(a.preprocessing, b.preprocessing)
        assert np.allclose(a.translation, b.translation) and np.allclose(a.quaternion_xyzw, b.quaternion_xyzw)
    s = str(tmp_path / "output_stats.txt")
    io.write_output_stats(s, 10000, 0, 0, 1.5, 0, 0.7, 1e9)
    st = io.read_output_stats(s)
    assert st["rendered"] == 10000 and st["runtime"] == 1.5 and st["icp_runtime"] == 0.7


def test_reference_demo_depth_png_unprojects():
    d = io.load_depth_png(os.path.join(G, "demo_depth.png"))
    assert d.shape == (480, 640) and d.max() == 51320
    xyz, pose, lab = oracle.depth_to_cloud(d, 8, 321.06398107, 242.97676897, 576.09757860, 576.09757860, 10000.0)
    sub = d[::8, ::8]
    assert len(xyz) == int((sub > 0).sum())
    assert np.allclose(np.sort(xyz[:, 2]), np.sort(sub[sub > 0].astype(np.float32) / np.float32(10000.0)))


def test_read_poses_txt_edge_cases(tmp_path):
    """One-pass parse for regular files, line-by-line otherwise: the first 7 fields of each line up to the
    first empty line (search_env.cpp:7098-7130 getline + stod), CRLF endings, trailing spaces, extra fields."""
    import numpy as np
    from perception_amd import io

    rng = np.random.default_rng(2)
    R = rng.normal(size=(6, 7))
    row = lambda r: " ".join(repr(float(v)) for v in r)  # noqa: E731
    cases = {
        "regular": ("\n".join(row(r) for r in R) + "\n", R),
        "crlf": ("\r\n".join(row(r) for r in R) + "\r\n", R),
        "trailing_space": ("\n".join(row(r) + " " for r in R) + "\n", R),
        "extra_fields": ("\n".join(row(np.append(r, 9.0)) for r in R) + "\n", R),
        "stops_at_empty_line": ("\n".join(row(r) for r in R[:3]) + "\n\n" + row(R[4]) + "\n", R[:3]),
        "no_final_newline": ("\n".join(row(r) for r in R), R),
        "empty": ("", np.zeros((0, 7))),
    }
    for name, (text, want) in cases.items():
        p = tmp_path / f"{name}.txt"
        p.write_text(text)
        got = io.read_poses_txt(str(p))
        assert got.shape == want.shape and np.array_equal(got, want), name


def test_read_poses_txt_cached_reparses_a_changed_file(tmp_path):
    from perception_amd import io as pio
    import os
    p = str(tmp_path / "poses.txt")
    rows = np.array([[0.1, 0.2, 0.3, 0.0, 0.0, 0.0, 1.0]])
    pio.write_poses_txt(p, rows)
    a = pio.read_poses_txt_cached(p)
    assert np.array_equal(a, pio.read_poses_txt(p)) and pio.read_poses_txt_cached(p) is a
    pio.write_poses_txt(p, np.vstack([rows, rows * 2]))
    os.utime(p, ns=(os.stat(p).st_atime_ns, os.stat(p).st_mtime_ns + 1000))
    b = pio.read_poses_txt_cached(p)
    assert b.shape == (2, 7) and not b.flags.writeable


def test_read_poses_txt_cached_same_size_same_mtime_rewrite(tmp_path):
    """A poses.txt rewritten in place with the same size and the same timestamps is parsed again (the cache is keyed
    by content); use_cache=False always parses."""
    from perception_amd import io as pio
    import os
    p = str(tmp_path / "poses.txt")
    rows = np.array([[0.1, 0.2, 0.3, 0.0, 0.0, 0.0, 1.0]])
    pio.write_poses_txt(p, rows)
    st = os.stat(p)
    a = pio.read_poses_txt_cached(p)
    pio.write_poses_txt(p, rows[:, [1, 0, 2, 3, 4, 5, 6]])  # same length: x and y swapped
    os.utime(p, ns=(st.st_atime_ns, st.st_mtime_ns))
    assert os.stat(p).st_size == st.st_size and os.stat(p).st_mtime_ns == st.st_mtime_ns
    b = pio.read_poses_txt_cached(p)
    assert b[0, 0] == 0.2 and a[0, 0] == 0.1
    assert pio.read_poses_txt_cached(p, use_cache=False) is not b
    for i in range(pio._POSES_CACHE_MAX + 5):  # LRU bound
        q = str(tmp_path / f"p{i}.txt")
        pio.write_poses_txt(q, rows * (i + 1))
        pio.read_poses_txt_cached(q)
    assert len(pio._POSES_CACHE) <= pio._POSES_CACHE_MAX


def test_read_poses_txt_cached_settled_file_skips_the_read(tmp_path, monkeypatch):
    """A file whose ctime was settled when it was read is served from its stat signature without reading the bytes
    again; rewriting it afterwards (same size, mtime put back) changes ctime, and the new content is parsed."""
    from perception_amd import io as pio
    import os
    import time
    p = str(tmp_path / "poses.txt")
    rows = np.array([[0.1, 0.2, 0.3, 0.0, 0.0, 0.0, 1.0]])
    pio.write_poses_txt(p, rows)
    st = os.stat(p)
    real_fs_now = pio._fs_now_ns
    monkeypatch.setattr(pio, "_fs_now_ns", lambda d, dev=None: real_fs_now(d, dev) + 10 * pio._SETTLED_NS)  # old file
    a = pio.read_poses_txt_cached(p)
    digests = []
    monkeypatch.setattr(pio, "_content_digest", lambda d: digests.append(1) or b"x" * 16)
    assert pio.read_poses_txt_cached(p) is a and not digests  # stat hit: nothing read or hashed
    time.sleep(0.05)  # past the coarse timestamp clock's tick
    pio.write_poses_txt(p, rows[:, [1, 0, 2, 3, 4, 5, 6]])
    os.utime(p, ns=(st.st_atime_ns, st.st_mtime_ns))
    assert os.stat(p).st_ctime_ns != st.st_ctime_ns
    monkeypatch.undo()
    b = pio.read_poses_txt_cached(p)
    assert b[0, 0] == 0.2 and a[0, 0] == 0.1


def test_read_poses_txt_cached_settles_on_the_file_systems_clock(tmp_path, monkeypatch):
    """"settled" is judged on the file system's clock (this host's plus an offset measured with a
    temporary file beside the file), so a local clock far ahead of the server's (NFS) does not make a fresh file look
    settled -- the step of the local clock is seen and the offset measured again."""
    from perception_amd import io as pio
    import time
    p = str(tmp_path / "poses.txt")
    pio.write_poses_txt(p, np.array([[0.1, 0.2, 0.3, 0.0, 0.0, 0.0, 1.0]]))
    pio._fs_now_ns(str(tmp_path))  # offset measured before the local clock steps
    real_ns = time.time_ns
    monkeypatch.setattr(pio.time, "time_ns", lambda: real_ns() + 100 * pio._SETTLED_NS)  # local clock far ahead
    a = pio.read_poses_txt_cached(p)
    digests = []
    real_digest = pio._content_digest
    monkeypatch.setattr(pio, "_content_digest", lambda d: digests.append(1) or real_digest(d))
    assert pio.read_poses_txt_cached(p) is a and digests  # fresh on the file system's clock: read and hashed again
    fs_now = pio._fs_now_ns(str(tmp_path))
    assert fs_now is not None and abs(fs_now - real_ns()) < 60 * 10**9


def test_fs_clock_offset_is_measured_once_per_device(tmp_path, monkeypatch):
    """one temporary file per device (and per 10 minutes), not one per read of a fresh file."""
    from perception_amd import io as pio
    calls = []
    real = pio._fs_clock_offset
    monkeypatch.setattr(pio, "_fs_clock_offset", lambda d: calls.append(d) or real(d))
    pio._FS_CLOCK.clear()
    p = str(tmp_path / "poses.txt")
    pio.write_poses_txt(p, np.array([[0.1, 0.2, 0.3, 0.0, 0.0, 0.0, 1.0]]))
    for _ in range(5):
        pio._POSES_STAT.clear()
        pio.read_poses_txt_cached(p)
    assert len(calls) == 1


def test_read_only_directory_settles_on_the_local_clock(tmp_path, monkeypatch):
    """where no temporary file can be created (a read-only data set) a file settles on this host's clock
    after 60 s instead of never (every search re-read and re-hashed every poses.txt)."""
    from perception_amd import io as pio
    import time
    p = str(tmp_path / "poses.txt")
    pio.write_poses_txt(p, np.array([[0.1, 0.2, 0.3, 0.0, 0.0, 0.0, 1.0]]))
    monkeypatch.setattr(pio, "_fs_clock_offset", lambda d: None)  # no temporary file possible
    pio._FS_CLOCK.clear()
    pio._POSES_STAT.clear()
    digests = []
    real_digest = pio._content_digest
    monkeypatch.setattr(pio, "_content_digest", lambda d: digests.append(1) or real_digest(d))
    pio.read_poses_txt_cached(p)
    pio.read_poses_txt_cached(p)
    assert len(digests) == 2  # fresh: hashed every time
    real_ns = time.time_ns
    monkeypatch.setattr(pio.time, "time_ns", lambda: real_ns() + 2 * pio._SETTLED_LOCAL_NS)  # a minute later
    pio._POSES_STAT.clear()
    pio.read_poses_txt_cached(p)
    pio.read_poses_txt_cached(p)
    assert len(digests) == 3  # settled after the first of these reads
