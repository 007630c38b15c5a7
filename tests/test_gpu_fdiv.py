"""pcore_fdiv.h (the fused kernel's division without range scaling) equals the compiler's IEEE f32
division bit for bit on the GPU: tools/fdiv_check.hip draws 134M (a, b) pairs over every exponent --
zeros, denormals, infinities, NaNs, a dense band around the fast path's [2^-40, 2^41) bounds and
quotients near rounding ties -- and counts mismatches; and that cvt_i32_rz_sat (v_cvt_i32_f32) has the
reference GPU's int32_t(float) semantics (round toward zero, saturate, NaN -> 0); and that the certified
fragment depth equals the IEEE one.  The binary is built by __graft_entry__.build()."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fdiv_exact_matches_ieee_division():
    exe = os.path.join(ROOT, "tools", "bin", "fdiv_check")
    if not os.path.exists(exe):
        pytest.fail("tools/bin/fdiv_check missing: run __graft_entry__.build()")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0 and res["mismatches"] == 0 and res["cvt_mismatches"] == 0, r.stdout + r.stderr
    assert 0.2 < res["fast_frac"] < 0.9  # both the fast path and the IEEE fallback are exercised


def test_certified_fragment_depth_matches_ieee():
    """frag_depth_certified (reciprocal estimates + an error certificate, IEEE divisions where it fails) gives the
    IEEE fragment depth bit for bit on ~1e9 inside-test barycentrics x vertex depths, many a few ulps from x.5."""
    exe = os.path.join(ROOT, "tools", "bin", "fdiv_check")
    if not os.path.exists(exe):
        pytest.fail("tools/bin/fdiv_check missing: run __graft_entry__.build()")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["frag_values"] > 10**8 and res["frag_mismatches"] == 0, r.stdout + r.stderr
    assert 0.2 < res["frag_certified_frac"] < 1.0  # certificate and IEEE fallback both exercised (the draw is
    # rich in out-of-range depths and half-integers, so most of it takes the fallback)
