"""Build libpcore.so (the HIP/gfx950 hot path + its C ABI) in-tree with hipcc.

The library is compiled with -ffp-contract=off so that every float expression keeps the reference's
explicit operation order (integer z-buffers bit-exact with the CPU oracle).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libpcore.so")
SOURCES = ["pcore_kernels.hip", "pcore_gicp.hip", "pcore_metrics.hip", "pcore_states.hip", "pcore_api.hip"]
HEADERS = ["pcore_internal.h", "pcore_cov.h", "pcore_gicp_math.h", "pcore_dmath.h", "pcore_colour.h", "pcore_fdiv.h", "pcore_streams.h", os.path.join("..", "..", "include", "pcore.h")]
ARCH = os.environ.get("PCORE_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: cannot build libpcore.so")


def flags() -> list:
    # -fno-slp-vectorize: the SLP vectorizer packs adjacent f32 adds / muls into v_pk_*_f32, which gfx950 issues at
    # half the rate of two plain VALU instructions' worth of issue slots plus extra register moves; without it the
    # fused COST kernel is 4.9 % faster (0.477 -> 0.454 ms per 10k C2 poses, same-box A/B; C3 unchanged).
    # -O2: the fused kernel schedules slightly differently than at -O3 (same registers, 6 waves per SIMD) and the C2
    # bench ran faster in 4 of 4 alternating pairs, 30.42 vs 30.04 M poses/s on average; C3 unchanged (25.6 / 25.5 ms
    # per step); the whole GPU suite green; -O1 / -Os / -O2 -fno-unroll-loops measured slower or equal (profiles/r03fl/).
    # The arithmetic is the same at any level (-ffp-contract=off, no fast-math).
    return [f"--offload-arch={ARCH}", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
            "-fno-fast-math", "-fno-slp-vectorize", "-Wall", "-Wno-unused-function"]


def kernel_source_digest() -> str:
    """SHA-256 (16 hex) of the compile flags and the sources that define the fused COST kernel: ties a committed
    counter profile (profiles/sq_counters.json) to the build it measured."""
    import hashlib

    h = hashlib.sha256(" ".join(flags()).encode())  # the compile flags too: a profile is of one build
    for f in ("pcore_kernels.hip", "pcore_internal.h", "pcore_cov.h", "pcore_colour.h", "pcore_fdiv.h", "pcore_streams.h"):
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def gicp_source_digest() -> str:
    """SHA-256 (16 hex) of the sources that define the GICP kernels: ties profiles/sq_counters_gicp.json to the code
    it measured."""
    import hashlib

    h = hashlib.sha256(" ".join(flags()).encode())
    for f in ("pcore_gicp.hip", "pcore_cov.h", "pcore_gicp_math.h", "pcore_dmath.h", "pcore_internal.h"):
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.abspath(__file__)]  # flags live here
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return LIB
    cmd = [hipcc()] + flags() + [os.path.join(CSRC, f) for f in SOURCES] + ["-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(LIB + ".tmp", LIB)
    return LIB


def build_checkers(verbose: bool = False) -> list:
    """Test-infrastructure binaries under tools/bin (not part of libpcore.so): fdiv_check compares
    pcore_fdiv.h's division against the compiler's IEEE division on the GPU (tests/test_gpu_fdiv.py)."""
    root = os.path.dirname(HERE)
    out_dir = os.path.join(root, "tools", "bin")
    os.makedirs(out_dir, exist_ok=True)
    built = []
    for name in ("fdiv_check",):
        src = os.path.join(root, "tools", name + ".hip")
        out = os.path.join(out_dir, name)
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", src,
               "-o", out]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True, cwd=root)
        built.append(out)
    return built


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
